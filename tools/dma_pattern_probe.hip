// Probe: HBM read rate of the bundle scan's access pattern -- per wave, rows
// of S slots x C bytes (16-byte buffer loads straight into LDS), the slots a
// read apart (12.5 KB, the uniform 50 kb layout), stepping C bytes a round
// through 32 * 848 / (S * C) ... -- with no compute: is 848-byte chunking
// what caps the scan's reads near 3.7 TB/s?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((address_space(3))) void* lds_ptr;

template <int S, int C>
__global__ void __launch_bounds__(256) k(const uint32_t* planes, uint64_t n_reads, uint64_t read_bytes,
                                          unsigned long long* queue, uint32_t* sink) {
  __shared__ uint32_t lds[4][8192];  // 32 KB a wave
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(unsigned long)(lds_ptr)lds[wv]);
  const uint64_t nb = n_reads / S;
  const int rounds = (int)(read_bytes / C);
  constexpr int kUnits = C / 16, kLoads = (kUnits + 63) / 64;
  uint32_t acc = 0;
  for (;;) {
    unsigned long long v = 0;
    if (lane == 0) v = atomicAdd(queue, 1ull);
    const uint64_t b = (uint64_t)__builtin_amdgcn_readfirstlane((int)v);
    if (b >= nb) break;
    const uint64_t off0 = b * S * read_bytes;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(reinterpret_cast<const char*>(planes) + off0), (short)0, (int)(S * read_bytes), 0x00020000);
    for (int r = 0; r < rounds; ++r) {
#pragma unroll
      for (int c = 0; c < kLoads; ++c) {
        if (64 * c + lane < kUnits) {
#pragma unroll
          for (int s = 0; s < S; ++s)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr)(unsigned long)(base + (s * kUnits + 64 * c) * 16 % 32768),
                                                     16, 16u * (64 * c + lane), (uint32_t)(s * read_bytes + (uint64_t)r * C), 0, 0);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      acc += lds[wv][lane];
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int S, int C>
void run(const uint32_t* planes, uint64_t n_reads, uint64_t read_bytes, unsigned long long* q, uint32_t* sink) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipMemset(q, 0, 8);
    (void)hipEventRecord(a);
    k<S, C><<<256, 256>>>(planes, n_reads, read_bytes, q, sink);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double bytes = (double)(n_reads / S * S) * (double)(read_bytes / C * C);
    if (rep == 2) printf("S=%2d slots x C=%5d B chunks: %.3f ms, %.2f TB/s\n", S, C, ms, bytes / ms / 1e9);
  }
}

int main() {
  const uint64_t n_reads = 640000, read_bytes = 12544;  // 50 kb reads: 12,544 bytes of planes a read
  uint32_t* planes;
  unsigned long long* q;
  uint32_t* sink;
  (void)hipMalloc(&planes, n_reads * read_bytes);
  (void)hipMemset(planes, 1, n_reads * read_bytes);
  (void)hipMalloc(&q, 8);
  (void)hipMalloc(&sink, 4);
  run<32, 848>(planes, n_reads, read_bytes, q, sink);
  run<16, 1696>(planes, n_reads, read_bytes, q, sink);
  run<8, 3392>(planes, n_reads, read_bytes, q, sink);
  run<32, 1024>(planes, n_reads, read_bytes, q, sink);
  run<4, 6272>(planes, n_reads, read_bytes, q, sink);
  return 0;
}
