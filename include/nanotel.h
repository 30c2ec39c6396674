/*
 * nanotel.h -- C-ABI of the MI355X-native NanoTel hot path.
 *
 * Drop-in boundary: one call per chunk replaces the per-chunk block of
 * NanoTel.R's run_future_worker_chuncks (NanoTel.R:2234-2256: the `< 8 reads`
 * sequential search_patterns call, or the 8 forked `%<-% search_patterns`
 * futures and their Reduce(union_all)), i.e. everything below
 * readDNAStringSet/reverseComplement and above write_csv:
 *
 *   reference interface (NanoTel.R)                  replaced by
 *   ------------------------------------------------ ----------------------------
 *   extract_patterns + fixed test   :2322-2334, :334 nt_compile
 *   reverseComplement(dna_reads)    :2219-2221       nt_params.rc (nt_pack_reads)
 *   analyze_subtelos / get_density_iranges / split_telo / get_sub_density
 *                                   :717-766, :308-397, :199-227, :449-468
 *                                                    nt_scan_call (window counts)
 *   find_telo_position_wraper and callees :1080-1155, :973-1077, :1692-1764,
 *                                   :843-959, :496-697   nt_scan_call (rows)
 *   analyze_read row logic          :1774-1862, :1920-1976 nt_scan_call (rows)
 *   search_patterns serials + 8-way split/union_all :2001-2078, :2234-2258
 *                                                    nt_assign_serials
 *
 * Conventions: plain pointers and sizes only; 0 = NT_OK, negative = error,
 * message via nt_last_error(ctx).  Positions are 1-based like IRanges; -1 is
 * the reference's "no telomere" sentinel (NA in summary.csv).  A context is
 * owned by one host thread.  HIP must not be initialised before a fork
 * (R future::multicore): create the context in the process that calls.
 */
#ifndef NANOTEL_H
#define NANOTEL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NT_OK 0
#define NT_E_ARG (-1)
#define NT_E_PATTERN (-2)     /* empty pattern ("empty pattern"), letter outside DNA_ALPHABET,
                                 or length > 18 (testit::assert NanoTel.R:589,647) */
#define NT_E_LETTER (-3)      /* read letter outside DNA_ALPHABET (readDNAStringSet errors) */
#define NT_E_EMPTY_READ (-4)  /* seq(1, 0, by=L) errors in split_telo (NanoTel.R:216) */
#define NT_E_RIGHT_EMPTY (-5) /* --check_right_edge on a read with no window (NanoTel.R:861) */
#define NT_E_NEG_WIDTH (-6)   /* IRanges(start, end) with end < start - 1 */
#define NT_E_HIP (-7)
#define NT_E_NOMEM (-8)
#define NT_E_LIMIT (-9)       /* > 64 patterns, TVR > 64 letters, subseq_length > 43690 */
#define NT_E_STATE (-10)      /* nt_compile() not called */
#define NT_E_IO (-11)         /* an output file could not be written */

/* summary flags per read */
#define NT_ROW_TELOMERIC 0x01 /* row emitted: max telomere width >= 30 (NanoTel.R:1847) */
#define NT_ROW_NA(p) (0x02 << (p)) /* pass p start == -1 -> NA columns (NanoTel.R:1926) */
#define NT_ROW_ERR_ALIGN 0x10 /* layout contract: blk_off[r] odd, or a bundle's planes more than 2 GiB apart;
                                 the read was skipped */
#define NT_ROW_DONE 0x80

typedef struct nt_ctx nt_ctx;

typedef struct {
  const char* patterns;      /* --patterns, whitespace separated (required) */
  const char* tvr_patterns;  /* --tvr_patterns or NULL */
  int32_t subseq_length;     /* --subseq_length (100) */
  double min_density;        /* --min_density (0.6) */
  int32_t check_right_edge;  /* --check_right_edge */
  int32_t rc;                /* --rc: reverse-complement every read before the scan */
  int32_t legacy_no_ext;     /* test switch: 2023 code without search_left/right_patterns */
} nt_params;

typedef struct {
  int32_t n_pass; /* 2 (exact, 1-mismatch) or 3 (+TVR) */
  int32_t n_pat;  /* unique() patterns */
  int32_t n_tvr;
  int32_t n_hits; /* hit counters per read: 2*n_pat + n_tvr */
  int32_t raw_p1; /* P1 keeps raw views (single fixed pattern) */
  int32_t jit;    /* 1: the scan runs as a kernel specialised for these patterns (hiprtc);
                     0: ahead-of-time kernels (NT_JIT=0 in the environment, or hiprtc failed) */
  int32_t tscan;  /* 1: bundled reads take the bundle scan (nt_tscan.h; NT_TSCAN=0 turns it off) */
  int32_t count_bytes; /* bytes per window count in win_counts: 1 (subseq_length <= 170) or 2 */
} nt_program_info;

/* Device-resident read batch (device pointers).  Layout: see DESIGN.md
 * "HBM layout": planes = uint2 {lo,hi} bit planes per 32 bases; read r owns
 * nt_read_blocks(len[r]) blocks from the even block index blk_off[r]. */
typedef struct {
  const uint32_t* planes;
  const uint64_t* blk_off;  /* [n_reads] first 32-base block of each read (even) */
  const uint32_t* len;      /* [n_reads] */
  const uint64_t* win_off;  /* [n_reads] prefix sum of the window ROWS nt_window_rows(nw) of the reads */
  const uint32_t* exc_off;  /* [n_reads+1] or NULL: non-ACGT letters */
  const uint32_t* exc_pos;
  const uint8_t* exc_code;
  uint64_t n_reads;
  uint64_t n_windows;       /* sum of the window rows (win_counts has n_windows*n_pass entries) */
  /* Bundle scan (optional): reads grouped 32 to a bundle
   * (nt_bundle_plan), scanned together from their own planes (no second copy
   * of the reads).  bnd_read == NULL or n_bundles == 0: every read takes the
   * per-read scan.  Else the bundled reads take the bundle scan and the reads
   * in list[0 .. n_list) the per-read scan (list may be NULL when n_list == 0).
   * A bundle's reads must lie within 2 GiB of planes of each other (what
   * nt_bundle_plan guarantees when given blk_off); the reads of a bundle that
   * does not are returned with NT_ROW_ERR_ALIGN. */
  const uint32_t* bnd_read;   /* [n_bundles * 32] read of each slot, ~0u = empty */
  uint64_t n_bundles;
  const uint32_t* list;       /* reads outside the bundles */
  uint64_t n_list;
} nt_batch;

/* Device-resident outputs (device pointers). */
typedef struct {
  void* win_counts;     /* [n_windows * n_pass] counts of count_bytes (uint8 / uint16): pass p of read r at
                           win_off[r]*n_pass + p*rows(r); 128-B aligned base */
  int32_t* start;       /* [n_reads*3] */
  int32_t* end;         /* [n_reads*3] */
  double* density;      /* [n_reads*3] */
  uint8_t* flags;       /* [n_reads] */
  uint32_t* hits;       /* [n_reads*n_hits] or NULL */
} nt_out;

typedef struct {
  uint64_t seed;
  uint64_t first_read;
  uint64_t read_len;
  double p_tract;       /* 0.5 */
  double sub_rate;      /* 0.02 */
  double variant_rate;  /* 0 (C2) / 0.05 (C3, C4) */
  uint32_t tract_min;   /* 1000 */
  uint32_t tract_max;   /* 15000 */
  int32_t rc_layout;    /* tract at the right end (for --rc configs) */
} nt_synth_params;

const char* nt_version(void);

/* --- context ------------------------------------------------------------ */
int nt_create(int device, nt_ctx** out);
void nt_destroy(nt_ctx* ctx);
const char* nt_last_error(const nt_ctx* ctx);
int nt_set_stream(nt_ctx* ctx, void* hip_stream); /* NULL = the context's own stream */
int nt_synchronize(nt_ctx* ctx);

/* --- A1: patterns and flags (extract_patterns NanoTel.R:2322-2334) ------- */
int nt_compile(nt_ctx* ctx, const nt_params* params, nt_program_info* info);

/* --- host packing (A14 reverseComplement fused when params.rc) ----------- */
int64_t nt_window_count(int64_t n, int32_t subseq_length);
/* The window-count row of a read and pass: nw rounded up to a multiple of 64
 * (whole 128-byte lines; the padding windows hold unspecified values). */
uint64_t nt_window_rows(int64_t nw);
/* 32-base blocks of a read's slot in the plane buffer: 2*ceil(n/64).  Slots
 * start at EVEN block offsets (the scan loads 64-base segments, 16 bytes). */
uint64_t nt_read_blocks(uint64_t n);
/* Pass 1: sizes.  Returns NT_E_LETTER (and *bad_read) on an invalid letter. */
int nt_pack_count(const char* const* seqs, const uint64_t* lens, uint64_t n_reads,
                  int32_t subseq_length, uint64_t* total_blocks, uint64_t* total_windows,
                  uint64_t* total_exc, uint64_t* max_len, uint64_t* bad_read);
/* Pass 2: fill host arrays sized by nt_pack_count (exc_* may be NULL when total_exc == 0). */
int nt_pack_reads(const char* const* seqs, const uint64_t* lens, uint64_t n_reads, int32_t rc,
                  int32_t subseq_length, uint32_t* planes, uint64_t* blk_off, uint32_t* len,
                  uint64_t* win_off, uint32_t* exc_off, uint32_t* exc_pos, uint8_t* exc_code);

/* --- bundles (the bundle scan's groups of reads) -------------------------- */
/* Host: which reads with non-ACGT letters must stay on the per-read scan.
 * The bundle scan takes reads with exceptions too: the calling kernel recounts
 * the windows within (longest pattern - 1) of an exception exactly, as it
 * recounts every bundled read's last window -- up to NT_EXC_WINDOWS (16) such
 * windows a read.  has_exc[r] = 1 for the reads with more (their exceptions
 * from nt_pack_reads: exc_off [n+1], exc_pos; exc_off NULL = none), 0 for the
 * rest: pass it to nt_bundle_plan.  Replaces no reference interface (the
 * reference has no bundles; Biostrings matches any subject, NanoTel.R:360-393). */
int nt_exc_marks(nt_ctx* ctx, const uint32_t* len, const uint32_t* exc_off, const uint32_t* exc_pos,
                 uint64_t n_reads, uint8_t* has_exc);
/* Host: group the reads of a batch 32 to a bundle (longest first; the compiled
 * program fixes the window size L).  has_exc (NULL = none) marks reads that
 * stay outside the bundles and go to the per-read scan: reads whose non-ACGT
 * letters reach too many windows (nt_exc_marks; marking every read with an
 * exception list is allowed too), or any the caller leaves there; so do the
 * reads of any program the bundle scan does not cover (then *n_bundles = 0).
 * blk_off (NULL = the caller vouches for it): the batch's block offsets; a
 * bundle whose reads' planes do not lie within 2 GiB of each other goes to the
 * per-read scan whole.  A read with exceptions in a bundle needs the batch's
 * exception lists in the nt_batch of nt_scan_call.  Outputs: bnd_read
 * [ceil(n/32)*32], list [n] (the reads left out, in order). */
int nt_bundle_plan(nt_ctx* ctx, const uint32_t* len, const uint64_t* blk_off, const uint8_t* has_exc,
                   uint64_t n_reads, uint32_t* bnd_read, uint64_t* n_bundles, uint32_t* list, uint64_t* n_list);

/* --- the hot path --------------------------------------------------------- */
/* Asynchronous on the context stream.  max_len = longest read of the batch. */
int nt_scan_call(nt_ctx* ctx, const nt_batch* batch, const nt_out* out, uint64_t max_len);

/* Pipelined batches (device-resident callers streaming batch after batch):
 * with on != 0 an nt_scan_call that runs the bundle scan in ranges returns
 * with its last range's calling still running on the library's calling
 * stream, beside the NEXT nt_scan_call's first scan range (the bundle scan is
 * bandwidth-bound, the calling latency-bound), instead of making the context
 * stream wait for it.  A batch's outputs are complete once nt_join (the
 * context stream waits for every calling launched so far) or nt_synchronize
 * has run.  Two consecutive calls must not share output buffers (the
 * library's own aux buffers alternate).  Turning it off joins.  The
 * reference processes its chunks one after another (NanoTel.R:2171-2268);
 * this only overlaps the device work of consecutive ones. */
int nt_set_pipelined(nt_ctx* ctx, int on);
/* Pipelined only: a call's INPUTS (planes, lengths, offsets, exception
 * lists and bundle lists) are read by its last calling kernel
 * after nt_scan_call returns, so they must not be overwritten (or freed) until
 * that calling is done.  nt_wait_call(ctx, back) makes the context stream wait
 * for the calling of the call `back` calls before the latest one (0 = the
 * latest, 1 = the one before); work enqueued on the context stream after it
 * may then overwrite that call's inputs.  A caller refilling ONE input set
 * waits with back = 0 before each refill; one alternating two input sets
 * waits with back = 1 (keeping the overlap).  Calls further back (back >= 2)
 * are already ordered on the context stream: each call's scans wait for the
 * calling of the call two before it.  nt_join waits for all of them. */
int nt_wait_call(nt_ctx* ctx, uint32_t back);
int nt_join(nt_ctx* ctx);

/* Measurement: with profiling on, every nt_scan_call records HIP events on
 * the context stream around its scan kernel(s) and its calling kernel.
 * nt_kernel_times waits for them and returns the summed spans of the calls
 * since the previous nt_kernel_times (or nt_set_profiling); returns the
 * number of calls, or < 0.  With the bundle scan in ranges (NT_TSUB), whose
 * calling kernels run beside the next range's scan on a second stream,
 * scan_ms sums the bundle-scan kernels' spans and call_ms is the remainder
 * of the call (the calling not hidden behind them). */
int nt_set_profiling(nt_ctx* ctx, int on);
int64_t nt_kernel_times(nt_ctx* ctx, double* scan_ms, double* call_ms);
/* Scan-kernel launches (bundle-scan ranges count one each) behind the last
 * nt_kernel_times: scan_ms / this = the scan kernel's average launch. */
int64_t nt_kernel_launches(const nt_ctx* ctx);
/* The calling kernels' own spans behind the last nt_kernel_times (events on
 * the stream each ran on, so a calling kernel hidden beside a scan range is
 * timed too): *call_ms = their sum; returns how many launches. */
int64_t nt_call_kernel_times(const nt_ctx* ctx, double* call_ms);
/* Calling-kernel launches since nt_create: out[0] ahead-of-time, out[1] the
 * specialised (hiprtc) kernel -- a benchmark checks that none of its timed
 * launches fell back to the ahead-of-time kernel. */
int nt_call_launch_counts(const nt_ctx* ctx, int64_t* out2);
/* 1 if the last nt_scan_call ran the calling kernel specialised for the
 * program's patterns (hiprtc; batches of >= 65,536 reads once it is built,
 * every batch with NT_CALL_JIT=1), 0 for the ahead-of-time one (same results). */
int nt_call_jit_state(const nt_ctx* ctx);
/* The first batch of >= 65,536 reads starts the hiprtc build of that
 * specialised calling kernel on a background thread (seconds; code objects are
 * kept in an on-disk cache, NT_JIT_CACHE); until it is done large batches run
 * the ahead-of-time kernel.  This starts it if need be and waits for it:
 * 1 = built, 0 = unavailable (the ahead-of-time kernel serves). */
int nt_call_jit_wait(nt_ctx* ctx);
/* Host only (no device): compile the kernels specialised for a parameter set
 * into the on-disk code-object cache (arch: "gfx950"), so that a later
 * nt_compile / first large batch loads them instead of running hiprtc. */
int nt_jit_prebuild(const nt_params* params, const char* arch);

/* Host-buffer convenience: pack (+rc), upload, scan+call, download, sync.
 * win_counts/hits optional.  Returns the first per-read error, if any. */
int nt_analyze_host(nt_ctx* ctx, const char* const* seqs, const uint64_t* lens, uint64_t n_reads,
                    int32_t* start, int32_t* end, double* density, uint8_t* flags,
                    void* win_counts, uint32_t* hits);

/* Host-path phase times of the context's nt_analyze_host calls (seconds,
 * cumulative): [0] layout of the batch, [1] 2-bit packing, [2] bundle plan,
 * [3] uploads enqueued, [4] device work + downloads, [5] row checks. */
int nt_host_times(const nt_ctx* ctx, double* t6);

/* --- --use_filter pre-filter ----------------------------------------------
 * Replaces filter_reads(samples, patterns, do_rc = FALSE, right_edge) +
 * filter_density (NanoTel.R:2083-2103, 2121-2163) as called per chunk from
 * run_future_worker_chuncks (NanoTel.R:2227-2232): keep[r] = 1 iff read r
 * (scan orientation) is >= 1e3 long and the union of the exact fixed=FALSE
 * matches of the patterns covers >= 0.8 * min_density of its 200-base edge
 * sub-read (subseq(start=71, width=200), or subseq(end=-71, width=200) with
 * check_right_edge).  The caller keeps the reads with keep = 1, in order.
 * nt_filter_call: device batch, keep = device [n_reads], asynchronous.
 * nt_filter_host: host reads (+rc as compiled), keep = host [n_reads], sync. */
int nt_filter_call(nt_ctx* ctx, const nt_batch* batch, uint8_t* keep);
int nt_filter_host(nt_ctx* ctx, const char* const* seqs, const uint64_t* lens, uint64_t n_reads,
                   uint8_t* keep);

/* --- A15: serials and row order of one chunk (host only) ----------------- */
/* Same contract as the reference: serial_start_io = this chunk's serial_start
 * (1.0 first), becomes max(Serial)+1; max_serial_io running max (-Inf first). */
int64_t nt_assign_serials(const uint8_t* is_telo, uint64_t n, double* serial_start_io,
                          double* max_serial_io, double* serial_out, int64_t* order_out);

/* --- analyze_read's rows as the columns of the summary data.frame --------- */
/* R's NA values, written where a pass found no telomere: NA_integer_ and the
 * NA_real_ NaN (payload 1954), so a .Call shim passes INTEGER() / REAL() of
 * its column vectors straight through. */
#define NT_NA_INT32 ((int32_t)0x80000000)
#define NT_NA_REAL_BITS 0x7FF00000000007A2ull
/* The rows of one chunk, row i = read order[i] (order/rows from
 * nt_assign_serials: the reference's group-major row order, NanoTel.R:2254),
 * as analyze_read's columns (NanoTel.R:1820-1837, 1926-1974):
 *   col_serial[i]  = serial[order[i]]                        Serial (double)
 *   col_length[i]  = lens[order[i]]                          sequence_length
 *   and per pass p < n_pass, at [p*rows + i]:
 *   col_density / col_start / col_end / col_width (= end - start + 1)
 *     -> telo_density, Telomere_start, Telomere_end, Telomere_length
 *        (suffixes "", "_mismatch", "_mismatch_tvr"); all four NA when the
 *        pass's start is -1 (NanoTel.R:1926-1940, 1956-1961).
 * sequence_ID is the caller's names[order[i]].  start/end/density: the
 * [n_reads*3] outputs of nt_scan_call / nt_analyze_host.  Returns rows or < 0
 * (NT_E_ARG: an order entry >= n_reads; NT_E_LIMIT: a read >= 2^31 bases). */
int64_t nt_rows_columns(const int32_t* start, const int32_t* end, const double* density,
                        const uint64_t* lens, uint64_t n_reads, int32_t n_pass,
                        const double* serial, const int64_t* order, int64_t rows,
                        double* col_serial, int32_t* col_length, double* col_density,
                        int32_t* col_start, int32_t* col_end, int32_t* col_width);

/* The same rows as text: summary.csv lines (write_csv, NanoTel.R:2430-2432;
 * readr's formatting restated -- shortest round-trip doubles, integral values
 * bare, NA, Inf, quoted names; sci_threshold > 0: integral Serials at or
 * above it as "<digits>e<zeros>", parity unpinned) and, when ids_out is given,
 * reads_ids.txt lines (write_lines, :2433).  names[i] / name_lens[i]: row i's
 * sequence_ID.  Returns the CSV bytes written (ids bytes in *ids_bytes), or
 * NT_E_LIMIT when a buffer is too small (2 * name + 3 + (3 + 4 n_pass) * 40
 * bytes a row always suffice). */
int64_t nt_rows_csv(const double* col_serial, const int32_t* col_length, const double* col_density,
                    const int32_t* col_start, const int32_t* col_end, const int32_t* col_width,
                    int64_t rows, int32_t n_pass, const char* const* names, const uint64_t* name_lens,
                    double sci_threshold, char* csv_out, uint64_t csv_cap, char* ids_out,
                    uint64_t ids_cap, uint64_t* ids_bytes);

/* --- host ingest: FASTA/FASTQ(.gz) in nrec-record chunks ------------------ */
/* readDNAStringSet(open_input_files(path), nrec, format) (NanoTel.R:2171-2216):
 * path = a file or a directory (files listed recursively, sorted, read as one
 * record stream); format 0 = fasta, 1 = fastq; gzip transparent.  A chunk's
 * names/sequences stay valid through the next nt_reader_next call (chunk k+1
 * may be read while chunk k is scanned; nt_reader_keep for more), or close.
 * Plain files are mapped and records point into them (no copies); gzip input
 * is inflated into shared windows; wrapped FASTA sequences are joined.
 * Returns the number of records (0 at the end) or < 0 (nt_reader_error). */
typedef struct nt_reader nt_reader;
int nt_reader_open(const char* path, int format, nt_reader** out);
void nt_reader_close(nt_reader* r);
uint64_t nt_reader_file_count(const nt_reader* r);
const char* nt_reader_file(const nt_reader* r, uint64_t i);
const char* nt_reader_error(const nt_reader* r);
int64_t nt_reader_next(nt_reader* r, uint64_t nrec, const char* const** names,
                       const uint64_t** name_lens, const char* const** seqs,
                       const uint64_t** seq_lens);
/* The next nrec records without copying them (a multi-GPU rank passing over
 * the chunks other ranks scan): the same parse and errors as nt_reader_next,
 * only the sequence lengths are kept (valid through the next nt_reader_skip;
 * a skip does not retire an nt_reader_next chunk). */
int64_t nt_reader_skip(nt_reader* r, uint64_t nrec, const uint64_t** seq_lens);
/* Keep the last `chunks` chunks valid (default 2, i.e. a chunk stays valid
 * through the next call): a caller that scans several chunks in one device
 * call holds them all.  Only grows. */
int nt_reader_keep(nt_reader* r, uint32_t chunks);

/* --- sharded ingest (one process per GPU; replaces every R worker reading the
 * whole chunk stream, NanoTel.R:2207-2254): each rank finds the chunk starts
 * from 1/N of the input and reads only its own chunks.  Chunk k is still
 * records [k nrec, (k+1) nrec) of the whole stream (A15 unchanged).
 * nt_reader_layout: file sizes and offsets in the concatenated stream;
 *   *all_plain = no file is gzip (then byte ranges shard it).
 * nt_reader_shard_range: the records that START in bytes [a, b) of the
 *   concatenated plain files (resynchronised at a FASTA '>' line / a FASTQ '@'
 *   line whose second next line starts with '+'); returns their count, with
 *   *first = the first record start parsed (>= a) and *next = the first start
 *   >= b (the total size at the end).  A caller checks first(rank r) ==
 *   next(rank r - 1): a mismatch means a false resynchronisation.
 * nt_reader_shard_positions: their global byte offsets (valid until the next call).
 * nt_reader_count_files: the record count of each listed file (whole files,
 *   on host threads; gzip parts of a run directory).
 * nt_reader_plan: before the first read -- the files this reader will visit,
 *   ascending (the inflate-ahead workers take only these).
 * nt_reader_seek: mode 0 = to byte a of the concatenated plain files (a record
 *   start); mode 1 = to record b of file a.  Seeks go forward in the plan.
 * nt_reader_stats: out[0] = bytes parsed (records read or skipped, index
 *   passes included), out[1] = bytes inflated. */
int nt_reader_layout(nt_reader* r, int* all_plain, uint64_t* total_bytes);
int64_t nt_reader_shard_range(nt_reader* r, uint64_t a, uint64_t b, uint64_t* first, uint64_t* next);
int64_t nt_reader_shard_positions(const nt_reader* r, const uint64_t** pos);
int nt_reader_count_files(nt_reader* r, const uint64_t* files, uint64_t n, uint64_t* counts);
int nt_reader_plan(nt_reader* r, const uint64_t* files, uint64_t n);
int nt_reader_seek(nt_reader* r, int mode, uint64_t a, uint64_t b);
int nt_reader_stats(const nt_reader* r, uint64_t* out2);

/* --- reads/<serial>.fasta.gz ---------------------------------------------
 * writeXStringSet(current_seq, "<output_dir>/reads/<serial>.fasta.gz",
 * compress = TRUE) for n telomeric reads (NanoTel.R:1869-1873): file i =
 * '>' names[i], then seqs[i] in 80-column lines (rc[i] != 0: its reverse
 * complement, Biostrings' letter pairs -- rc may be NULL), gzip as R's
 * gzfile() writes it (deflate level `level`, R's default 6; mtime 0, OS 3).
 * The files are written by `threads` host threads (<= 0: the library's
 * default, at most 16, divided by LOCAL_WORLD_SIZE).  Returns NT_OK, or
 * NT_E_IO with *err_index = the first read whose file failed (NT_E_LIMIT: a
 * read of 4 Gbases or more). */
int nt_write_fasta_gz(const char* const* paths, const char* const* names, const uint64_t* name_lens,
                      const char* const* seqs, const uint64_t* seq_lens, const uint8_t* rc, uint64_t n,
                      int32_t level, int32_t threads, uint64_t* err_index);

/* --- synthetic long reads (bench / tests) --------------------------------- */
int nt_synth_device(nt_ctx* ctx, const nt_synth_params* sp, uint64_t n_reads, uint32_t* planes_dev);
int nt_uniform_layout_device(nt_ctx* ctx, uint64_t n_reads, uint64_t read_len, int32_t subseq_length,
                             uint64_t* blk_off_dev, uint32_t* len_dev, uint64_t* win_off_dev);
int nt_synth_ascii(const nt_synth_params* sp, uint64_t read_index, char* out);
/* --rc for a device-resident batch: planes_out read r = reverseComplement of
 * planes_in read r (NanoTel.R:2219-2221), the same blk_off / len; out of place,
 * asynchronous on the context stream.  Reads must be A/C/G/T only (a batch with
 * non-ACGT letters takes the host packer, nt_pack_reads rc = 1). */
int nt_rc_device(nt_ctx* ctx, const uint32_t* planes_in, uint32_t* planes_out, const uint64_t* blk_off_dev,
                 const uint32_t* len_dev, uint64_t n_reads);

#ifdef __cplusplus
}
#endif
#endif
