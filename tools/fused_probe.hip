// fused_probe.hip -- what a bundle scan that reads the per-read planes
// directly (no T-layout copy) would pay, on MI355X.
//
// The bundle scan walks lane = window (block of L positions), bit = slot of a
// 32-read bundle.  Reading the per-read planes instead of the T-layout means
// each lane fetches, per range of 32 positions of its block, one new 8-byte
// plane word {lo, hi} of each of the 32 reads, extracts the 32-position piece
// at its block's bit offset (v_alignbit) and transposes the 32 x 32 bit
// matrices (lo and hi) in its own registers.  Variants:
//   0: contiguous 16-byte streaming of the same bytes (the copy ceiling)
//   1: the per-range word loads only (one range ahead), xor-consumed
//   2: 1 + extraction + lane-local transposes
//   3: 2 + a synthetic walk of ~20 VALU per position
// usage: fused_probe [n_reads] [read_len]
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

constexpr int kL = 100, kLam = 6;
constexpr int kNR = (kL + 2 * kLam + 31) / 32;  // ranges of 32 positions per block

template <int I, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    sfor<I + 1, N>(f);
  }
}

// a[k] bit p = M[k][p]  ->  a[p] bit k = M[k][p] (32 x 32, in registers)
__device__ __forceinline__ void transpose32(uint32_t (&a)[32]) {
  // byte stages by v_perm: j = 16, 8
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t x = a[k], y = a[k + 16];
    a[k] = __builtin_amdgcn_perm(y, x, 0x05040100u);       // lo16(x) | lo16(y) << 16
    a[k + 16] = __builtin_amdgcn_perm(y, x, 0x07060302u);  // hi16(x) | hi16(y) << 16
  }
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    if (k & 8) continue;
    const uint32_t x = a[k], y = a[k + 8];
    a[k] = __builtin_amdgcn_perm(y, x, 0x06020400u);      // x0 y0 x2 y2
    a[k + 8] = __builtin_amdgcn_perm(y, x, 0x07030501u);  // x1 y1 x3 y3
  }
  sfor<0, 3>([&](auto ji) {
    constexpr int j = 4 >> decltype(ji)::value;
    constexpr uint32_t m = j == 4 ? 0x0F0F0F0Fu : j == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      if (k & j) continue;
      const uint32_t x = a[k], y = a[k + j];
      a[k] = (x & m) | ((y << j) & ~m);
      a[k + j] = ((x >> j) & m) | (y & ~m);
    }
  });
}

__global__ void __launch_bounds__(256) k_stream(const uint4* __restrict__ in, uint64_t n16, unsigned* sink) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x, T = gridDim.x * 256ull;
  uint32_t acc = 0;
  uint4 r[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = t + T * i < n16 ? in[t + T * i] : make_uint4(0, 0, 0, 0);
  for (uint64_t i = t; i < n16; i += 8 * T) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint4 v = r[j];
      const uint64_t nx = i + T * (8 + j);
      r[j] = nx < n16 ? in[nx] : make_uint4(0, 0, 0, 0);
      acc ^= v.x + v.y * 3 + v.z * 5 + v.w * 7;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int V>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
k_fused(const uint2* __restrict__ planes, uint64_t W, uint64_t n_bundles, int nblk, unsigned long long* queue,
        unsigned* sink) {
  const int lane = threadIdx.x & 63;
  uint32_t acc = 0;
  for (;;) {
    unsigned long long v = 0;
    if (lane == 0) v = atomicAdd(queue, 1ull);
    const uint64_t b = (uint64_t)__builtin_amdgcn_readfirstlane((int)v);
    if (b >= n_bundles) break;
    const uint2* base = planes + b * 32 * W;
    const int nst = (nblk + 63) / 64;
    for (int st = 0; st < nst; ++st) {
      const int k = st * 64 + lane;
      const int pos0 = k * kL - kLam;
      const int q0 = pos0 >> 5;
      const uint32_t sh = (uint32_t)(pos0 & 31);
      const int qmax = (int)W - 1;
      auto ld = [&](int s, int q) -> uint2 {
        q = q < 0 ? 0 : (q > qmax ? qmax : q);
        return base[(uint64_t)s * W + q];
      };
      uint2 carry[32], nxt[32];
#pragma unroll
      for (int s = 0; s < 32; ++s) carry[s] = ld(s, q0);
#pragma unroll
      for (int s = 0; s < 32; ++s) nxt[s] = ld(s, q0 + 1);
#pragma unroll
      for (int r = 0; r < kNR; ++r) {
        uint2 fut[32];
        if (r + 1 < kNR) {
#pragma unroll
          for (int s = 0; s < 32; ++s) fut[s] = ld(s, q0 + r + 2);
        }
        if constexpr (V == 1) {
#pragma unroll
          for (int s = 0; s < 32; ++s) acc ^= nxt[s].x * (s + 1) + nxt[s].y;
        } else {
          uint32_t pl[32], ph[32];
#pragma unroll
          for (int s = 0; s < 32; ++s) {
            pl[s] = __builtin_amdgcn_alignbit(nxt[s].x, carry[s].x, sh);
            ph[s] = __builtin_amdgcn_alignbit(nxt[s].y, carry[s].y, sh);
          }
          transpose32(pl);
          transpose32(ph);
          if constexpr (V == 2) {
#pragma unroll
            for (int p = 0; p < 32; ++p) acc ^= pl[p] + ph[p];
          } else {
            // synthetic walk: ~20 VALU per position over a short history
            uint32_t h0 = acc, h1 = acc ^ 1u, h2 = acc ^ 2u, c0 = 0, c1 = 0;
#pragma unroll
            for (int p = 0; p < 32; ++p) {
              const uint32_t L_ = pl[p], H_ = ph[p];
              const uint32_t tT = L_ & H_, tA = ~(L_ | H_), tG = ~L_ & H_;
              const uint32_t a3 = __builtin_amdgcn_bitop3_b32(tT, h0, h1, 0x80);
              const uint32_t m3 = __builtin_amdgcn_bitop3_b32(tA, h1, h2, 0xE8);
              const uint32_t x1 = __builtin_amdgcn_bitop3_b32(a3, m3, tG, 0xE8);
              const uint32_t x2 = __builtin_amdgcn_bitop3_b32(x1, h0, tT, 0xFE);
              const uint32_t x3 = __builtin_amdgcn_bitop3_b32(x2, h2, a3, 0xFE);
              const uint32_t s0 = __builtin_amdgcn_bitop3_b32(c0, x3, x1, 0x96);
              const uint32_t s1 = __builtin_amdgcn_bitop3_b32(c0, x3, x1, 0xE8);
              const uint32_t u0 = __builtin_amdgcn_bitop3_b32(c1, s1, x2, 0x96);
              const uint32_t u1 = __builtin_amdgcn_bitop3_b32(c1, s1, x2, 0xE8);
              const uint32_t y0 = __builtin_amdgcn_bitop3_b32(u0, m3, tA, 0x96);
              const uint32_t y1 = __builtin_amdgcn_bitop3_b32(u1, a3, tG, 0xE8);
              const uint32_t y2 = __builtin_amdgcn_bitop3_b32(y0, y1, h1, 0xFE);
              const uint32_t y3 = __builtin_amdgcn_bitop3_b32(y2, x2, h0, 0x96);
              const uint32_t y4 = __builtin_amdgcn_bitop3_b32(y3, y1, s0, 0xE8);
              h2 = h1;
              h1 = h0;
              h0 = __builtin_amdgcn_bitop3_b32(tT, tA, y4, 0x96);
              c0 = s0 ^ y4;
              c1 = u1 | y3;
            }
            acc ^= h0 + h1 + h2 + c0 + c1;
          }
        }
        if (r + 1 < kNR) {
#pragma unroll
          for (int s = 0; s < 32; ++s) {
            carry[s] = nxt[s];
            nxt[s] = fut[s];
          }
        }
      }
      if (k >= nblk) acc = 0;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// lane (l, h) = half h of window 32 st + l: walk starts at window start + h L/2 - kLam
template <int V>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1)))
k_half(const uint2* __restrict__ planes, uint64_t W, uint64_t n_bundles, int nblk, unsigned long long* queue,
       unsigned* sink) {
  constexpr int kNR2 = (kL / 2 + 2 * kLam + 31) / 32;
  const int lane = threadIdx.x & 63, l = lane & 31, h = lane >> 5;
  uint32_t acc = 0;
  for (;;) {
    unsigned long long v = 0;
    if (lane == 0) v = atomicAdd(queue, 1ull);
    const uint64_t b = (uint64_t)__builtin_amdgcn_readfirstlane((int)v);
    if (b >= n_bundles) break;
    const uint2* base = planes + b * 32 * W;
    const int nst = (nblk + 31) / 32;
    for (int st = 0; st < nst; ++st) {
      const int k = st * 32 + l;
      const int pos0 = k * kL + h * (kL / 2) - kLam;
      const int q0 = pos0 >> 5;
      const uint32_t sh = (uint32_t)(pos0 & 31);
      const int qmax = (int)W - 1;
      auto ld = [&](int s, int q) -> uint2 {
        q = q < 0 ? 0 : (q > qmax ? qmax : q);
        return base[(uint64_t)s * W + q];
      };
      uint2 carry[32], nxt[32];
#pragma unroll
      for (int s = 0; s < 32; ++s) carry[s] = ld(s, q0);
#pragma unroll
      for (int s = 0; s < 32; ++s) nxt[s] = ld(s, q0 + 1);
#pragma unroll
      for (int r = 0; r < kNR2; ++r) {
        uint2 fut[32];
        if (r + 1 < kNR2) {
#pragma unroll
          for (int s = 0; s < 32; ++s) fut[s] = ld(s, q0 + r + 2);
        }
        if constexpr (V == 1) {
#pragma unroll
          for (int s = 0; s < 32; ++s) acc ^= nxt[s].x * (s + 1) + nxt[s].y;
        } else {
          uint32_t pl[32], ph[32];
#pragma unroll
          for (int s = 0; s < 32; ++s) {
            pl[s] = __builtin_amdgcn_alignbit(nxt[s].x, carry[s].x, sh);
            ph[s] = __builtin_amdgcn_alignbit(nxt[s].y, carry[s].y, sh);
          }
          transpose32(pl);
          transpose32(ph);
#pragma unroll
          for (int p = 0; p < 32; ++p) acc ^= pl[p] + ph[p];
        }
        if (r + 1 < kNR2) {
#pragma unroll
          for (int s = 0; s < 32; ++s) {
            carry[s] = nxt[s];
            nxt[s] = fut[s];
          }
        }
      }
      if (k >= nblk) acc = 0;
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// is a buffer load's soffset part of the raw-buffer range check?  records =
// 256 bytes; lane i loads voffset 4 i with soffset 128: lanes 32..63 read
// bytes 256.. (out of range if soffset counts), lanes 0..31 bytes 128..255
__global__ void k_soff(const uint32_t* p, uint32_t* out) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(p), (short)0, 256, 0x00020000);
  out[threadIdx.x] = __builtin_amdgcn_raw_buffer_load_b32(rs, 4 * threadIdx.x, 128, 0);
}

int main(int argc, char** argv) {
  {
    uint32_t *p, *o;
    CK(hipMalloc(&p, 4096));
    CK(hipMalloc(&o, 256));
    std::vector<uint32_t> h(1024);
    for (int i = 0; i < 1024; ++i) h[i] = 1000 + i;
    CK(hipMemcpy(p, h.data(), 4096, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_soff, dim3(1), dim3(64), 0, 0, p, o);
    CK(hipMemcpy(h.data(), o, 256, hipMemcpyDeviceToHost));
    std::printf("soffset range check: lane 0 -> %u (word 32 = 1032), lane 31 -> %u, lane 32 -> %u (0 if soffset "
                "is range-checked, 1064 if not), lane 63 -> %u\n", h[0], h[31], h[32], h[63]);
  }
  const uint64_t n_reads = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 500000;
  const uint64_t len = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 50000;
  const uint64_t W = 2 * ((len + 63) / 64);  // uint2 words per read
  const uint64_t nb = n_reads / 32;
  const int nblk = (int)((len + kL - 1) / kL);
  const uint64_t bytes = n_reads * W * 8;
  uint2* planes;
  CK(hipMalloc(&planes, bytes));
  {
    std::vector<uint32_t> h(1 << 24);
    uint32_t x = 12345;
    for (auto& v : h) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; v = x; }
    for (uint64_t o = 0; o < bytes; o += h.size() * 4)
      CK(hipMemcpy((char*)planes + o, h.data(), std::min<uint64_t>(h.size() * 4, bytes - o), hipMemcpyHostToDevice));
  }
  unsigned* sink;
  unsigned long long* q;
  CK(hipMalloc(&sink, 4));
  CK(hipMalloc(&q, 8));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    float best = 1e30f, sum = 0.f;
    for (int it = 0; it < 7; ++it) {
      CK(hipMemset(q, 0, 8));
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (it >= 2) { best = std::min(best, ms); sum += ms; }
    }
    std::printf("%-34s best %.3f ms mean %.3f ms  %.2f TB/s of planes (%.2f GB)\n", name, best, sum / 5,
                bytes / (best * 1e-3) / 1e12, bytes / 1e9);
  };
  timeit("0 contiguous 16-B stream", [&] {
    hipLaunchKernelGGL(k_stream, dim3(cus * 8), dim3(256), 0, 0, (const uint4*)planes, bytes / 16, sink);
  });
  timeit("1 per-range word loads", [&] {
    hipLaunchKernelGGL(k_fused<1>, dim3(cus), dim3(256), 0, 0, planes, W, nb, nblk, q, sink);
  });
  timeit("2 + extract + transpose", [&] {
    hipLaunchKernelGGL(k_fused<2>, dim3(cus), dim3(256), 0, 0, planes, W, nb, nblk, q, sink);
  });
  timeit("3 + synthetic walk (~20/pos)", [&] {
    hipLaunchKernelGGL(k_fused<3>, dim3(cus), dim3(256), 0, 0, planes, W, nb, nblk, q, sink);
  });
  timeit("4 half-window lanes, loads", [&] {
    hipLaunchKernelGGL(k_half<1>, dim3(cus), dim3(256), 0, 0, planes, W, nb, nblk, q, sink);
  });
  timeit("5 half-window lanes + transpose", [&] {
    hipLaunchKernelGGL(k_half<2>, dim3(cus), dim3(256), 0, 0, planes, W, nb, nblk, q, sink);
  });
  timeit("6 = 1 at 2 waves/CU", [&] {
    hipLaunchKernelGGL(k_fused<1>, dim3(cus), dim3(128), 0, 0, planes, W, nb, nblk, q, sink);
  });
  timeit("7 = 4 at 2 waves/CU", [&] {
    hipLaunchKernelGGL(k_half<1>, dim3(cus), dim3(128), 0, 0, planes, W, nb, nblk, q, sink);
  });
  CK(hipGetLastError());
  return 0;
}
