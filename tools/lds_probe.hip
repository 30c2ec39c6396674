// Probe: 16-byte buffer loads straight into LDS (buffer_load_dwordx4 ... lds)
// on gfx950.  (1) layout: lane l's 16 bytes land at the LDS base + 16 l.
// (2) visibility: after s_waitcnt vmcnt(0), a ds_read of the same wave sees
// the loaded data -- checked over many cold loads (a large buffer, each
// iteration a fresh stretch), with an optional extra s_waitcnt lgkmcnt(0).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
typedef __attribute__((address_space(3))) void* lds_ptr;

__global__ void layout_k(const uint32_t* in, uint32_t* out, int n) {
  __shared__ uint32_t lds[64 * 4 * 3];
  for (int i = threadIdx.x; i < 64 * 4 * 3; i += 64) lds[i] = 0xDEADBEEF;
  __syncthreads();
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(in), (short)0, n * 4, 0x00020000);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr)(lds + 64 * 4), 16, (63 - threadIdx.x) * 16, 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 4 * 3; i += 64) out[i] = lds[i];
}

template <int kExtra>
__global__ void __launch_bounds__(256) vis_k(const uint32_t* in, uint64_t n_words, uint32_t* bad, int iters) {
  __shared__ uint32_t lds[4][64 * 4];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t* my = lds[wv];
  const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(unsigned long)(lds_ptr)my);
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(in), (short)0, 0x7FFFFFF0, 0x00020000);
  uint32_t nb = 0;
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + wv, nwaves = (uint64_t)gridDim.x * 4;
  for (int it = 0; it < iters; ++it) {
    const uint64_t chunk = (gw + nwaves * it) % (n_words / 256);  // 256 words = 1 KB a wave
    const uint32_t vo = (uint32_t)(chunk * 1024) + 16u * lane;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr)(unsigned long)base, 16, vo, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (kExtra) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // read a neighbour lane's unit (not the lane's own)
    const int l2 = (lane * 7 + 3) & 63;
    const uint4 v = *reinterpret_cast<const uint4*>(my + 4 * l2);
    const uint32_t w0 = (uint32_t)(chunk * 256) + 4u * l2;
    nb += (v.x != w0) + (v.y != w0 + 1) + (v.z != w0 + 2) + (v.w != w0 + 3);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the read is done before the next load
  }
  if (nb) atomicAdd(bad, nb);
}

int main() {
  uint32_t *in, *out, *bad;
  int n = 256;
  (void)hipMalloc(&in, n * 4);
  (void)hipMalloc(&out, 64 * 4 * 3 * 4);
  uint32_t h[256];
  for (int i = 0; i < n; ++i) h[i] = i;
  (void)hipMemcpy(in, h, n * 4, hipMemcpyHostToDevice);
  layout_k<<<1, 64>>>(in, out, n);
  uint32_t o[768];
  (void)hipMemcpy(o, out, sizeof(o), hipMemcpyDeviceToHost);
  int bl = 0, b0 = 0;
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 4; ++j)
      if (o[256 + 4 * l + j] != (uint32_t)(4 * (63 - l) + j)) ++bl;
  for (int i = 0; i < 256; ++i) b0 += (o[i] != 0xDEADBEEF) + (o[512 + i] != 0xDEADBEEF);
  printf("layout: bad %d, guard bad %d\n", bl, b0);
  // visibility over 1 GiB of words (value = word index)
  const uint64_t nw = 1ull << 28;
  uint32_t* big;
  (void)hipMalloc(&big, nw * 4);
  std::vector<uint32_t> hv(1 << 24);
  for (uint64_t c = 0; c < nw; c += hv.size()) {
    for (size_t i = 0; i < hv.size(); ++i) hv[i] = (uint32_t)(c + i);
    (void)hipMemcpy(big + c, hv.data(), hv.size() * 4, hipMemcpyHostToDevice);
  }
  (void)hipMalloc(&bad, 4);
  for (int extra = 0; extra < 2; ++extra) {
    (void)hipMemset(bad, 0, 4);
    if (extra) vis_k<1><<<1024, 256>>>(big, nw, bad, 64);
    else vis_k<0><<<1024, 256>>>(big, nw, bad, 64);
    uint32_t hb = 0;
    (void)hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
    printf("visibility (extra lgkmcnt wait %d): %u bad words of %llu\n", extra, hb, 1024ull * 4 * 64 * 64 * 4);
  }
  return 0;
}
