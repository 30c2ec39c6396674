#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void k(const uint32_t* in, uint32_t* out, int n) {
  __shared__ uint32_t lds[64 * 4 * 3];
  for (int i = threadIdx.x; i < 64 * 4 * 3; i += 64) lds[i] = 0xDEADBEEF;
  __syncthreads();
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(in), (short)0, n * 4, 0x00020000);
  // lane l loads 16 B from in[4*(63-l)] (reversed) into LDS unit k=1
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds + 64 * 4), 16, (63 - threadIdx.x) * 16, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 4 * 3; i += 64) out[i] = lds[i];
}
int main() {
  uint32_t *in, *out; int n = 256;
  hipMalloc(&in, n * 4); hipMalloc(&out, 64 * 4 * 3 * 4);
  uint32_t h[256]; for (int i = 0; i < n; ++i) h[i] = i;
  hipMemcpy(in, h, n * 4, hipMemcpyHostToDevice);
  k<<<1, 64>>>(in, out, n);
  uint32_t o[768]; hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) for (int j = 0; j < 4; ++j) if (o[256 + 4 * l + j] != (uint32_t)(4 * (63 - l) + j)) ++bad;
  int bad0 = 0; for (int i = 0; i < 256; ++i) { if (o[i] != 0xDEADBEEF) ++bad0; if (o[512 + i] != 0xDEADBEEF) ++bad0; }
  printf("lds dma b128: bad %d, guard bad %d, o[256..263] = %u %u %u %u %u %u %u %u\n", bad, bad0, o[256], o[257], o[258], o[259], o[260], o[261], o[262], o[263]);
  return bad || bad0;
}
