// rw_mix_bench.hip -- what a read stream pays for a small share of writes on
// MI355X (the bundle scan reads 6.84 GB and writes 0.69 GB per launch).
// Each wave streams its share of a read buffer with 16-byte loads (8 in
// flight per lane, like the scan's ring) and, every `every` iterations,
// stores 16 bytes per lane to a write buffer (plain or non-temporal).
// usage: rw_mix_bench [read_GB] ; prints one line per variant
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// waves stride over 1 KB "slots" (64 lanes x 16 B); a wave takes slots
// w, w + W, w + 2W, ...; writes: one 1 KB store per `every` slots (nt: non-temporal)
template <bool kNt>
__global__ void __launch_bounds__(256) rw(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t slots,
                                          int every, uint64_t wslots, unsigned* sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6), W = (uint64_t)gridDim.x * 4;
  uint32_t acc = 0;
  uint4 ring[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t s = w + W * i;
    ring[i] = s < slots ? in[s * 64 + lane] : make_uint4(0, 0, 0, 0);
  }
  uint64_t k = 0, wk = w;
  for (uint64_t s = w; s < slots; s += 8 * W) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint4 v = ring[i];
      const uint64_t sn = s + W * (8 + i);
      ring[i] = sn < slots ? in[sn * 64 + lane] : make_uint4(0, 0, 0, 0);
      acc ^= v.x + v.y * 3 + v.z * 5 + v.w * 7;
      if (every > 0 && ++k % every == 0) {
        const uint64_t d = (wk % wslots) * 64 + lane;
        wk += W;
        const u32x4 x = {acc, acc + 1, acc + 2, acc + 3};
        if (kNt)
          __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(out + d));
        else
          *reinterpret_cast<u32x4*>(out + d) = x;
      }
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// dedicated writer waves: blocks of 5 waves, waves 0-3 stream the reads (no
// stores), wave 4 writes its block's share of the stores, paced by s_sleep
__global__ void __launch_bounds__(320) rw_split(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                uint64_t slots, uint64_t writes_per_block, uint64_t wslots,
                                                unsigned* sink) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (wv == 4) {
    for (uint64_t i = 0; i < writes_per_block; ++i) {
      const uint64_t d = ((blockIdx.x + (uint64_t)gridDim.x * i) % wslots) * 64 + lane;
      const u32x4 x = {(unsigned)i, 1u, 2u, 3u};
      __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(out + d));
      __builtin_amdgcn_s_sleep(8);
    }
    return;
  }
  const uint64_t w = (uint64_t)blockIdx.x * 4 + wv, W = (uint64_t)gridDim.x * 4;
  uint32_t acc = 0;
  uint4 ring[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t s = w + W * i;
    ring[i] = s < slots ? in[s * 64 + lane] : make_uint4(0, 0, 0, 0);
  }
  for (uint64_t s = w; s < slots; s += 8 * W) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint4 v = ring[i];
      const uint64_t sn = s + W * (8 + i);
      ring[i] = sn < slots ? in[sn * 64 + lane] : make_uint4(0, 0, 0, 0);
      acc ^= v.x + v.y * 3 + v.z * 5 + v.w * 7;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? std::atof(argv[1]) : 6.84;
  const uint64_t slots = (uint64_t)(gb * 1e9 / 1024.0);
  const uint64_t wslots = slots / 4;
  uint4 *in, *out;
  unsigned* sink;
  CK(hipMalloc(&in, slots * 1024));
  CK(hipMalloc(&out, wslots * 1024));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(in, 1, slots * 1024));
  CK(hipMemset(out, 0, wslots * 1024));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct V {
    int every, nt, bpc;
  };
  std::vector<V> vs = {{0, 0, 1}, {10, 1, 1}, {10, 0, 1}, {200, 1, 1}, {1000, 1, 1}, {0, 0, 2}, {10, 1, 2}};
  // writes into a 4 MB region (L2-resident): the store acks come from L2
  for (const uint64_t ws : {wslots, (uint64_t)4096}) {
    for (const V& v : vs) {
      if (ws != wslots && (v.every == 0 || v.bpc != 1)) continue;
    const int grid = cus * v.bpc;
    float best = 1e30f;
    for (int it = 0; it < 6; ++it) {
      CK(hipEventRecord(a));
      if (v.nt)
        rw<true><<<grid, 256>>>(in, out, slots, v.every, ws, sink);
      else
        rw<false><<<grid, 256>>>(in, out, slots, v.every, ws, sink);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, a, b));
      if (it > 0 && ms < best) best = ms;
    }
    const double rd = slots * 1024.0, wr = v.every ? rd / v.every : 0.0;
    std::printf("every %4d nt %d blocks/CU %d region %s: %.3f ms  read %.2f GB  write %.3f GB  -> read %.2f TB/s\n",
                v.every, v.nt, v.bpc, ws == wslots ? "full" : "4MB ", best, rd / 1e9, wr / 1e9, rd / best / 1e9);
    }
  }
  {  // dedicated writer waves (0.68 GB of writes beside a read-only stream)
    const uint64_t wpb = slots / 10 / cus;
    float best = 1e30f, wbest = 0.f;
    for (int it = 0; it < 6; ++it) {
      CK(hipEventRecord(a));
      rw_split<<<cus, 320>>>(in, out, slots, wpb, wslots, sink);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, a, b));
      if (it > 0 && ms < best) best = ms;
    }
    for (int it = 0; it < 3; ++it) {  // the writer waves alone
      CK(hipEventRecord(a));
      rw_split<<<cus, 320>>>(in, out, 0, wpb, wslots, sink);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&wbest, a, b));
    }
    std::printf("writer waves: %.3f ms (writers alone %.3f ms)  read %.2f GB write %.3f GB -> read %.2f TB/s\n", best,
                wbest, slots * 1024.0 / 1e9, wpb * cus * 1024.0 / 1e9, slots * 1024.0 / best / 1e9);
  }
  return 0;
}
