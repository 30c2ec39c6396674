// Probe: where does a buffer load into LDS (buffer_load_dwordx4 ... lds) put
// its data when the instruction's immediate offset is not zero, and which
// global bytes does it read?  One wave loads 64 x 16 bytes from a source of
// word i = 1000 + i with M0 = the LDS buffer and offset:imm = 848 (one bundle
// slot row), soffset 0, voffset = 16 lane; the LDS words are dumped.
//   hipcc --offload-arch=gfx950 -O2 tools/lds_dma_probe.hip -o /tmp/lds_dma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                   \
      return 1;                                                             \
    }                                                                       \
  } while (0)

constexpr int kWords = 2048;  // 8 KB of LDS

template <int kImm>
__global__ void __launch_bounds__(64) k_probe(const uint32_t* src, uint32_t* out) {
  __shared__ uint32_t lds[kWords];
  for (int i = threadIdx.x; i < kWords; i += 64) lds[i] = 0xFFFFFFFFu;
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(src), (short)0,
                                                                        kWords * 4, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, 16u * threadIdx.x, 0,
                                           kImm, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < kWords; i += 64) out[i] = lds[i];
}

template <int kImm>
static int run(const uint32_t* src, uint32_t* out) {
  hipLaunchKernelGGL(k_probe<kImm>, dim3(1), dim3(64), 0, 0, src, out);
  CK(hipGetLastError());
  std::vector<uint32_t> h(kWords);
  CK(hipMemcpy(h.data(), out, kWords * 4, hipMemcpyDeviceToHost));
  int first = -1, last = -1;
  for (int i = 0; i < kWords; ++i)
    if (h[i] != 0xFFFFFFFFu) {
      if (first < 0) first = i;
      last = i;
    }
  std::printf("imm %4d: LDS words written %d..%d (bytes %d..%d); word %d = %u (source word %u); word %d = %u\n", kImm,
              first, last, 4 * first, 4 * last + 3, first, first >= 0 ? h[first] : 0u,
              first >= 0 ? h[first] - 1000u : 0u, last, last >= 0 ? h[last] : 0u);
  return 0;
}

int main() {
  uint32_t *src, *out;
  CK(hipMalloc(&src, kWords * 4));
  CK(hipMalloc(&out, kWords * 4));
  std::vector<uint32_t> h(kWords);
  for (int i = 0; i < kWords; ++i) h[i] = 1000 + i;
  CK(hipMemcpy(src, h.data(), kWords * 4, hipMemcpyHostToDevice));
  if (run<0>(src, out) || run<848>(src, out) || run<2544>(src, out) || run<4080>(src, out)) return 1;
  std::printf("(LDS address = M0 + imm + 16 lane if the words written start at imm; the source word then says "
              "whether imm also moves the global address)\n");
  return 0;
}
