// nt_rng.h -- counter-based synthetic long-read generator (host and device).
//
// Every base is a pure function of (seed, read index, position), so the GPU
// generator (nt_synth_kernel) and the host generator (nt_synth_ascii) produce
// identical reads without any shared state.  Workload:
//   * uniform ACGT background;
//   * with probability p_tract a read carries a telomeric tract of length
//     U[tract_min, tract_max] (clamped to the read) of (TTAGGG)n at its left
//     edge, each repeat unit replaced by TCAGGG/CTAGGG with probability
//     variant_rate and each base substituted with probability sub_rate;
//   * rc_layout: the read is the reverse complement of such a read (tract of
//     CCCTAA at the right end), so that `--rc` puts it back on the left.
#pragma once
#include <stdint.h>

#if defined(HIP_INCLUDE_HIP_HIP_RUNTIME_H)  // with the HIP runtime: host and device
#define NT_HD __host__ __device__ __forceinline__
#else
#define NT_HD static inline
#endif

struct NtSynth {
  uint64_t seed;
  uint64_t first_read;    // global index of the first read generated
  uint64_t read_len;
  uint32_t p_tract_u24;   // probability * 2^24
  uint32_t sub_u24;
  uint32_t variant_u24;
  uint32_t tract_min, tract_max;
  int32_t rc_layout;
};

struct NtSynthRead {
  uint32_t has_tract;
  uint64_t tract_len;
};

NT_HD uint64_t nt_mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

NT_HD uint64_t nt_read_key(uint64_t seed, uint64_t r) { return nt_mix64(seed ^ nt_mix64(2 * r + 1)); }

NT_HD NtSynthRead nt_synth_read(const NtSynth& S, uint64_t r) {
  const uint64_t h = nt_mix64(nt_read_key(S.seed, r) ^ 0x5A5A5A5A5A5A5A5Aull);
  NtSynthRead R;
  R.has_tract = (uint32_t)(h & 0xFFFFFFu) < S.p_tract_u24;
  const uint64_t span = (uint64_t)S.tract_max - S.tract_min + 1;
  uint64_t tl = S.tract_min + ((h >> 32) % span);
  if (tl > S.read_len) tl = S.read_len;
  R.tract_len = R.has_tract ? tl : 0;
  return R;
}

// 2-bit code (A=0 C=1 G=2 T=3) of base `pos` of the left-tract layout.
NT_HD uint32_t nt_synth_base_left(const NtSynth& S, const NtSynthRead& R, uint64_t key, uint64_t pos) {
  if (pos < R.tract_len) {
    // TTAGGG / TCAGGG / CTAGGG units
    const uint64_t unit = pos / 6, off = pos - unit * 6;
    const uint64_t hv = nt_mix64(key ^ (unit * 0xD1B54A32D192ED03ull + 0x1234567ull));
    uint32_t u = 0;  // 0 TTAGGG, 1 TCAGGG, 2 CTAGGG
    if ((uint32_t)(hv & 0xFFFFFFu) < S.variant_u24) u = 1u + (uint32_t)((hv >> 24) & 1u);
    // packed 2-bit codes, base 0 in the low bits (selects, not a local array:
    // a runtime-indexed array would live in scratch on the GPU)
    const uint32_t kTTAGGG = 3u | (3u << 2) | (0u << 4) | (2u << 6) | (2u << 8) | (2u << 10);
    const uint32_t kTCAGGG = 3u | (1u << 2) | (0u << 4) | (2u << 6) | (2u << 8) | (2u << 10);
    const uint32_t kCTAGGG = 1u | (3u << 2) | (0u << 4) | (2u << 6) | (2u << 8) | (2u << 10);
    const uint32_t unit_code = u == 0 ? kTTAGGG : (u == 1 ? kTCAGGG : kCTAGGG);
    uint32_t b = (unit_code >> (2 * off)) & 3u;
    const uint64_t hs = nt_mix64(key ^ (pos * 0x9E6C63D0676A9A99ull + 0xABCDEFull));
    if ((uint32_t)(hs & 0xFFFFFFu) < S.sub_u24) b = (uint32_t)((hs >> 24) & 3u);
    return b;
  }
  return (uint32_t)(nt_mix64(key ^ (pos * 0xA24BAED4963EE407ull)) & 3u);
}

NT_HD uint32_t nt_synth_base(const NtSynth& S, const NtSynthRead& R, uint64_t r, uint64_t pos) {
  const uint64_t key = nt_read_key(S.seed, r);
  if (S.rc_layout) return 3u - nt_synth_base_left(S, R, key, S.read_len - 1 - pos);
  return nt_synth_base_left(S, R, key, pos);
}
