// nt_common.h -- structures shared by the host library and the gfx950 kernels.
//
// HBM layout of a read batch ("bit-plane 2-bit packing"):
//   planes[b] = {lo, hi} (two uint32) for the 32-base block b; bit i of lo/hi is
//   the low/high bit of the 2-bit code of base 32*b+i (A=0 C=1 G=2 T=3).
//   Read r occupies the slot of 2*ceil(len[r]/64) blocks starting at the EVEN
//   block blk_off[r] (the scan loads 64-base segments = 16 bytes); bits past
//   the read end are don't-care (the kernels mask them).  Letters other than A/C/G/T (N, IUPAC
//   ambiguity codes, '-', '+', '.') are stored as A in the planes and listed in
//   a per-read exception list (position, Biostrings DNA code) -- see
//   DESIGN.md "Exceptions".
// Window counts: uint8 (L <= 170: every window, the widened last one too, is
//   under 256 bases -- NtProgram::cnt8) or uint16 at
//   win_counts[win_off[r]*n_pass + p*NT_WIN_ROWS(nw(r)) + i]
//   (covered bases of window i of pass p; nw = split_telo window count).  A
//   read's rows are padded to a multiple of 64 windows and win_off[r] is the
//   prefix sum of the PADDED counts, so every 64-window block of a row is one
//   128-byte line (the scans store whole lines: a partly written line costs a
//   read-modify-write in the memory system) and 16-byte aligned for the bundle
//   scan's 8-count stores; the padding windows [nw, NT_WIN_ROWS(nw)) hold
//   unspecified values.
#pragma once
#ifndef __HIPCC_RTC__
#include <stdint.h>
#endif

#define NT_MAX_PAT 64     // unique patterns per list (--patterns / --tvr_patterns)
#define NT_MAX_M 18       // testit::assert(str_length(pattern) <= 18), NanoTel.R:589,647
#define NT_MAX_TVR_M 64   // TVRs: two overflow words per segment / neighbourhood word (nt_scan.h, nt_call.h)
#define NT_MAX_PASS 3
#define NT_WIN_ROWS(nw) (((nw) + 63) & ~63ull)  // windows of a padded count row

// Scan read queues (see scan_reads): per launch, NT_QUEUES u64 counters
// NT_QUEUE_STRIDE u64 apart (own 256-byte line each), zeroed before the launch
#define NT_QUEUES 8
#define NT_QUEUE_STRIDE 32
#define NT_QUEUE_WORDS (NT_QUEUES * NT_QUEUE_STRIDE)

// Per-read flag bits (rows.flags)
#define NT_FLAG_TELOMERIC 0x01   // row emitted (max width >= 30), NanoTel.R:1847-1868
#define NT_FLAG_NA_SHIFT 1       // bit 1+p: pass p start == -1 (NA columns)
#define NT_FLAG_ERR_ALIGN 0x10   // blk_off[r] odd: segments must be 16-byte aligned
#define NT_FLAG_ERR_RIGHT 0x20   // find_right_telo on a 0-row window table (R errors)
#define NT_FLAG_ERR_WIDTH 0x40   // IRanges(start, end) with negative width (R errors)
#define NT_FLAG_DONE 0x80        // the kernel processed this read

// One compiled pattern.  tt_scan[j]: 4-bit truth table over subject bases
// A,C,G,T (bit c) for matchPattern(fixed = <regex test>) in
// get_density_iranges; tt_eq[j]: the same for fixed=TRUE (code equality), used
// by the edge-extension steps (NanoTel.R:502-566, 614, 676 call matchPattern
// with the default fixed=TRUE).
struct NtPat {
  int32_t m;
  int32_t fixed;               // !str_detect(pat, "[WSMKRYBDHVN]")
  uint8_t code[NT_MAX_TVR_M];  // Biostrings DNA codes (for exception positions)
  uint8_t tt_scan[NT_MAX_TVR_M];
  uint8_t tt_eq[NT_MAX_TVR_M];
  // the truth tables expanded to bit-select masks (0 or ~0) for bases A,C,G,T:
  // loaded with scalar loads into SGPRs, so the match of a letter costs three
  // v_bfi_b32 and no decode
  uint32_t tm_scan[NT_MAX_TVR_M][4];
  uint32_t tm_eq[NT_MAX_TVR_M][4];
  // one-hot fast path (every letter a single base under the scan semantics):
  // letter j matches base (l,h) iff ((L ^ xl[j]) & (H ^ xh[j])) is set, with
  // xl = l ? 0 : ~0, xh = h ? 0 : ~0 -- two ops (v_xor + v_bitop3) per letter
  int32_t onehot;
  uint32_t xl[NT_MAX_TVR_M];
  uint32_t xh[NT_MAX_TVR_M];
};

struct NtProgram {
  int32_t n_pat, n_tvr;   // unique() lists
  int32_t n_pass;         // 2, or 3 with --tvr_patterns
  int32_t raw_p1;         // P1 keeps raw views: single fixed pattern (NanoTel.R:349-355)
  int32_t L;              // --subseq_length
  int32_t right_edge;     // --check_right_edge
  int32_t legacy_no_ext;  // test switch: skip search_left/right_patterns (2023 code)
  int32_t n_hits;         // 2*n_pat + n_tvr hit counters per read
  double min_density;     // --min_density
  uint64_t div_m;         // floor(p / L) = (p * div_m) >> div_s for p < 2^31 (exact)
  uint32_t div_s;
  uint32_t div32_m;       // floor(p / L) = umulhi(p, div32_m) >> div32_s, p < 2^31, L >= 2
  uint32_t div32_s;
  uint32_t thr_size;      // entries of the per-width telomeric threshold table
  int32_t cnt8;           // window counts are uint8 (L <= 170), else uint16
  int32_t m_max;          // longest pattern or TVR
  NtPat pat[NT_MAX_PAT];
  NtPat tvr[NT_MAX_PAT];
};

#if defined(__HIPCC_RTC__) || defined(__HIP__)
#define NT_HOSTDEV __host__ __device__
#else
#define NT_HOSTDEV
#endif

// Reads with a few non-ACGT letters take the bundle scan too.  The T-layout
// holds A at their exception positions, so a window holding a position within
// m_max - 1 of one may be counted wrong there; the calling kernel recounts
// those windows exactly from the read's planes and exception list
// (call_fix_windows, nt_call.h), as it recounts every bundled read's last
// window.  A read whose exceptions reach more than NT_EXC_WINDOWS windows
// before its last stays on the per-read scan (nt_exc_marks -> nt_bundle_plan).
#define NT_EXC_WINDOWS 16

// The windows before the last (nw - 1) that hold a position within mm - 1 of
// an exception (positions ascending), in order: f(w) for each of the first
// cap; returns how many there are, or cap + 1 when there are more.
template <class F>
NT_HOSTDEV inline int exc_windows(const uint32_t* pos, uint32_t n_exc, int n, int L, int nw, int mm, int cap, F&& f) {
  int cnt = 0, next = 0;  // next: the first window not visited yet
  for (uint32_t i = 0; i < n_exc && next < nw - 1; ++i) {
    const int p = (int)pos[i];
    const int a = p - (mm - 1) < 0 ? 0 : p - (mm - 1);
    const int b = p + (mm - 1) > n - 1 ? n - 1 : p + (mm - 1);
    int w0 = a / L, w1 = b / L;
    if (w1 > nw - 2) w1 = nw - 2;
    if (w0 < next) w0 = next;
    for (int w = w0; w <= w1; ++w) {
      if (cnt == cap) return cap + 1;
      ++cnt;
      f(w);
    }
    if (w1 + 1 > next) next = w1 + 1;
  }
  return cnt;
}

// Bundles (the bundle scan, nt_tscan.h): reads grouped NT_BUNDLE to a
//   bundle, slots sorted by length (non-increasing; read index ~0u = empty
//   slot), scanned together from their own planes: bnd_read[b * NT_BUNDLE + s].
#define NT_BUNDLE 32

struct NtBatch {
  const uint32_t* planes;   // uint2 blocks
  const uint64_t* blk_off;  // [n_reads]
  const uint32_t* len;      // [n_reads]
  const uint64_t* win_off;  // [n_reads] prefix sum of window counts
  const uint32_t* exc_off;  // [n_reads+1] or nullptr (no exceptions in batch)
  const uint32_t* exc_pos;  // sorted per read, 0-based positions
  const uint8_t* exc_code;  // Biostrings DNA codes
  uint64_t n_reads;
  // per-read scan (scan_reads): the reads it scans, list[i] (nullptr: all n_reads)
  const uint32_t* list;
  uint64_t n_list;
  // bundle scan (nt_tscan.h); n_bundles == 0: no bundles
  const uint32_t* bnd_read;    // [n_bundles * NT_BUNDLE]
  uint64_t n_bundles;
};

struct NtOut {
  void* win_counts;      // uint8 or uint16 (cnt8), see layout above
  int32_t* start;        // [n_reads*3], 1-based, -1 = NA
  int32_t* end;          // [n_reads*3]
  double* density;       // [n_reads*3]
  uint8_t* flags;        // [n_reads]
  uint32_t* hits;        // [n_reads*n_hits] or nullptr
};
