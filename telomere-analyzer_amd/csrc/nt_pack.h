// nt_pack.h -- host-only helpers shared by nt_host.cpp and nt_pack.cpp.
#pragma once
#include <stdint.h>
#include <stdlib.h>

#include <string>
#include <thread>
#include <vector>

#include "nanotel.h"
#include "nt_common.h"
#include "nt_rng.h"

namespace nt_host {

uint8_t letter_code(unsigned char c);  // Biostrings DNA_ALPHABET code, 0 = not a DNA letter
int64_t window_count(int64_t n, int L);  // split_telo windows (NanoTel.R:199-227)
inline uint64_t read_blocks(uint64_t n) { return 2 * ((n + 63) / 64); }  // 32-base blocks of a read's slot
// The program of a parameter set: patterns, passes, divisor magic, the
// telomeric threshold table (host only).
int make_program(const nt_params* prm, NtProgram& P, std::vector<uint32_t>& thr, std::string& err);
// The planes of one read (reverse-complemented when rc); non-ACGT letters are
// A in the planes and, with exc_pos, listed.  Returns their number, -1 for a
// letter outside DNA_ALPHABET.
int64_t pack_one(const unsigned char* s, uint64_t n, int rc, uint32_t* out, uint32_t* exc_pos, uint8_t* exc_code);
NtSynth to_synth(const nt_synth_params* sp);

// Host worker threads: this rank's share of the machine's (one process per
// GPU: the cores divided among the node's ranks), at most 16 (a GPU's share
// of the host on the MI355X nodes)
inline unsigned pool_threads() {
  unsigned nt = std::thread::hardware_concurrency();
  if (nt == 0) nt = 1;
  if (const char* w = std::getenv("LOCAL_WORLD_SIZE")) {
    const int k = std::atoi(w);
    if (k > 1) nt = nt / (unsigned)k > 0 ? nt / (unsigned)k : 1u;
  }
  return nt > 16u ? 16u : nt;
}

template <class F>
void parallel_for(uint64_t n, F&& f) {
  const unsigned nt = pool_threads();
  if (n < 64 || nt == 1) {
    for (uint64_t i = 0; i < n; ++i) f(i);
    return;
  }
  std::vector<std::thread> th;
  const uint64_t chunk = (n + nt - 1) / nt;
  for (unsigned t = 0; t < nt; ++t) {
    const uint64_t lo = t * chunk, hi = n < lo + chunk ? n : lo + chunk;
    if (lo >= hi) break;
    th.emplace_back([lo, hi, &f] {
      for (uint64_t i = lo; i < hi; ++i) f(i);
    });
  }
  for (auto& x : th) x.join();
}

}  // namespace nt_host
