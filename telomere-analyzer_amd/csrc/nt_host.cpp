// nt_host.cpp -- the C-ABI of include/nanotel.h: pattern compilation (A1),
// host packing (+ reverse complement, A14), launches of the gfx950 kernels,
// serial assignment (A15) and the synthetic-read generator.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "nanotel.h"
#include "nt_common.h"
#include "nt_rng.h"
#include "nt_pack.h"

extern "C" {
uint32_t nt_dev_wave_words(int single, int n_hits, int np, uint32_t nw_cap);
uint64_t nt_dev_tmask_words(uint64_t total_windows, uint64_t n_reads, int np);
hipError_t nt_dev_launch(const NtProgram* prog, const uint32_t* thr, const NtBatch* B,
                         const NtOut* O, uint64_t* tmask, unsigned long long* queue,
                         uint32_t len_lo, uint32_t len_hi, uint32_t claim, uint32_t nstatic,
                         int single, int one, int m6, int lds, uint32_t wave_words, uint32_t* gscr,
                         int grid, hipStream_t stream);
hipError_t nt_dev_set_lds_limit(uint32_t bytes);
int nt_dev_scan_blocks_per_cu(int single, int one, int m6, int lds, size_t lds_bytes);
hipError_t nt_dev_launch_call(const NtProgram* prog, const NtBatch* B, const NtOut* O,
                              const uint64_t* tmask, const uint32_t* thr, uint32_t thr_size, int fix_last,
                              int long_tvr, int call_grid, hipStream_t stream);
hipError_t nt_dev_launch_synth(const NtSynth* S, uint32_t* planes, uint64_t n_reads,
                               hipStream_t stream);
hipError_t nt_dev_launch_rc(const uint32_t* in, uint32_t* out, const uint64_t* blk_off, const uint32_t* len,
                            uint64_t n_reads, int cu_count, hipStream_t stream);
hipError_t nt_dev_launch_filter(const NtProgram* prog, const NtBatch* B, uint8_t* keep,
                                uint32_t thr_count, int right_edge, int grid, hipStream_t stream);
hipError_t nt_dev_launch_uniform_layout(uint64_t n_reads, uint64_t nblk, uint64_t read_len,
                                        uint64_t nw, uint64_t* blk_off, uint32_t* len,
                                        uint64_t* win_off, hipStream_t stream);
}

int nt_jit_blocks_per_cu(void* fn, size_t lds_bytes);
int nt_jit_block_threads(void* fn);
bool nt_jit_get(int device, const NtProgram& P, void* fn[4], void** tfn, std::string& err);
bool nt_tscan_eligible(const NtProgram& P);
hipError_t nt_tjit_launch(void* fn, int grid, hipStream_t stream, const NtBatch* B, const NtOut* O,
                          uint64_t* tmask, unsigned long long* queue, uint32_t thr_full);
void* nt_cjit_get(int device, const NtProgram& P, std::string& err);
int nt_jit_prebuild_program(const NtProgram& P, const std::string& arch);
hipError_t nt_cjit_launch(void* h, int np, int cu_count, hipStream_t stream, const NtProgram* prog,
                          const NtBatch* B, const NtOut* O, const uint64_t* tmask, const uint32_t* thr,
                          uint32_t thr_size, int fix_last);
hipError_t nt_jit_launch(void* fn, int grid, size_t lds_bytes, hipStream_t stream,
                         const NtProgram* prog, const uint32_t* thr, const NtBatch* B,
                         const NtOut* O, uint64_t* tmask, unsigned long long* queue,
                         uint32_t len_lo, uint32_t len_hi, uint32_t claim, uint32_t nstatic, uint32_t wave_words, uint32_t* gscr);

using namespace nt_host;

namespace {

constexpr uint32_t kLdsCapBytes = 64 * 1024;  // per 4-wave workgroup; longer reads: global scratch

// Process-wide pool of pinned host buffers: pinning (hipHostMalloc) costs
// milliseconds per 100 MB, so the staging of a destroyed context serves the
// next one (up to kMax bytes kept; never freed at exit, after HIP's teardown).
struct PinnedPool {
  static constexpr size_t kMax = 16ull << 30;
  std::mutex mu;
  std::vector<std::pair<void*, size_t>> free;
  size_t bytes = 0;
  void* take(size_t want, size_t& cap) {
    std::lock_guard<std::mutex> lk(mu);
    size_t best = free.size();
    for (size_t i = 0; i < free.size(); ++i)
      if (free[i].second >= want && (best == free.size() || free[i].second < free[best].second)) best = i;
    if (best == free.size()) return nullptr;
    void* p = free[best].first;
    cap = free[best].second;
    bytes -= cap;
    free.erase(free.begin() + (ptrdiff_t)best);
    return p;
  }
  void give(void* p, size_t cap) {
    {
      std::lock_guard<std::mutex> lk(mu);
      if (bytes + cap <= kMax) {
        free.emplace_back(p, cap);
        bytes += cap;
        return;
      }
    }
    (void)hipHostFree(p);
  }
};
PinnedPool& pinned_pool() {
  static PinnedPool* p = new PinnedPool;
  return *p;
}

// Pinned host staging (hipHostMalloc), kept across calls: no page faults or
// zero-fill per call and the uploads are DMA from page-locked memory.
struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) pinned_pool().give(p, cap);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes + bytes / 4, 4096);  // some headroom for the next chunk
    if ((p = pinned_pool().take(bytes, cap))) return hipSuccess;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  ~HostBuf() {
    if (p) pinned_pool().give(p, cap);
  }
};

// Device buffers in physically contiguous HBM (hipDeviceMallocContiguous),
// hipMalloc when that fails: the scans stream the planes, the T-layout and the
// counts from a thousand places at once, and on a box whose HBM is fragmented
// plain hipMalloc memory is mapped with small pages -- the c50k bundle scan ran
// 1.53 ms a range there instead of 1.38 (profiles/r04/contig/).  NT_DEV_CONTIG=0:
// hipMalloc only.
static bool dev_contig() {
  static const bool on = [] {
    const char* v = std::getenv("NT_DEV_CONTIG");
    return !(v && v[0] == '0');
  }();
  return on;
}
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(bytes, 256);
    hipError_t e = hipErrorOutOfMemory;
    if (want >= (64u << 20) && dev_contig()) e = hipExtMallocWithFlags(&p, want, hipDeviceMallocContiguous);
    if (e != hipSuccess) {
      (void)hipGetLastError();  // (a failed contiguous request leaves the error state set)
      p = nullptr;
      e = hipMalloc(&p, want);
    }
    if (e == hipSuccess) cap = want;
    return e;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
};

}  // namespace

struct nt_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  bool compiled = false;
  bool lds_limit_set = false;
  hipStream_t call_stream = nullptr;  // sub-batched calling kernels (NT_SUBBATCH > 1)
  hipEvent_t ev_scan = nullptr, ev_call = nullptr;
  // pipelined batches (nt_set_pipelined): a call leaves its last range's
  // calling on call_stream, beside the next call's first scan range; calls
  // alternate between two aux buffers (tmask / tmask_alt), and call i waits
  // for the calling of call i - 2 (ev_done[i % 2]) before its scan writes
  bool pipelined = false;
  uint64_t pipe_i = 0;
  hipEvent_t ev_done[2] = {nullptr, nullptr};
  bool profile = false;  // HIP events around the scan and call kernels of every call
  // per recorded call: [0] start, [1] end of the scans (serial calling), [2]
  // end, [3 + 2k], [4 + 2k] around bundle-scan range k (overlapped calling)
  static constexpr int kMaxTsub = 16;
  std::vector<std::array<hipEvent_t, 3 + 2 * (kMaxTsub + 1)>> ev;  // + the per-read scan of list reads
  std::vector<int> ev_nt;  // bundle-scan ranges of each recorded call
  int64_t last_launches = 0;  // scan-kernel launches of the last nt_kernel_times window
  // the calling kernels' own spans (events on the stream each runs on) of the
  // recorded calls: per call up to kMaxTsub + 1 launches
  std::vector<std::array<hipEvent_t, 2 * (kMaxTsub + 2)>> cev;
  std::vector<int> cev_n;
  double last_call_ms = 0.0;      // their sum over the last nt_kernel_times window
  int64_t last_call_launches = 0;
  int64_t call_launches[2] = {0, 0};  // calling launches since nt_create: [0] ahead-of-time, [1] specialised
  size_t n_ev = 0;  // calls recorded since the last nt_kernel_times
  bool jit = false;  // hiprtc-specialised scan kernels (nt_jit.cpp)
  void* jit_fn[4] = {};  // [no hit counters ? 2 : 0] + [global scratch ? 1 : 0]
  void* tjit_fn = nullptr;  // the bundle scan of the program (nt_tscan.h), or null
  std::vector<uint32_t> thr_h;  // telomeric threshold per window width (nt_compile)
  int tscan_bpc = 0;        // its resident 256-thread blocks per CU
  std::string jit_err;
  // the calling kernel specialised for the program (nt_call.h via hiprtc),
  // built on the first batch that uses it; null: the ahead-of-time kernel
  void* cjit_fn = nullptr;
  bool cjit_tried = false;
  // its build, started in the background by nt_compile (hiprtc, or the disk cache)
  std::future<std::pair<void*, std::string>> cjit_build;
  int cjit_last = 0;  // the last nt_scan_call launched it
  std::string cjit_err;
  NtProgram prog{};
  nt_params params{};
  NtProgram* prog_dev = nullptr;
  int cu_count = 256;
  DevBuf planes, blk_off, len, win_off, exc_off, exc_pos, exc_code;
  DevBuf wc, start, end, dens, flags, hits, scratch, tmask, thr, queue;
  DevBuf tmask_alt;  // the odd calls' aux buffer in pipelined mode
  DevBuf bnd_read, list;  // upload_reads' bundles
  HostBuf h_planes, h_meta;  // upload_reads staging
  // host-path phase times (s, cumulative; nt_host_times): layout, pack,
  // bundle plan, uploads, the device work and downloads, the row checks
  double host_t[6] = {};
};

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int fail(nt_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

// The calling kernel for a batch of n_reads: the hiprtc-specialised one
// (letter tests as constant truth tables; 117 VGPRs and no spills against the
// ahead-of-time kernel's 168 + 15 spilled) for batches of at least
// kCallJitMinReads reads -- its build takes ~20 s once per pattern set, which
// only a large batch repays -- else the ahead-of-time kernel (same results).
// NT_CALL_JIT=1 uses it for every batch, NT_CALL_JIT=0 never.
constexpr uint64_t kCallJitMinReads = 1u << 16;

static int call_jit_mode() {
  const char* v = std::getenv("NT_CALL_JIT");
  return v ? std::atoi(v) : -1;
}

// The specialised calling kernel of the program: its build (hiprtc, or the
// on-disk code-object cache) runs on a background thread, started by the first
// batch that would use it; returns false while it runs (waits when `wait`).
static bool cjit_collect(nt_ctx* ctx, bool wait) {
  if (ctx->cjit_tried) return true;
  if (!ctx->cjit_build.valid()) {
    const int dev = ctx->device;
    const NtProgram prog = ctx->prog;
    ctx->cjit_build = std::async(std::launch::async, [dev, prog]() {
      (void)hipSetDevice(dev);  // the module loads on this thread's device
      std::string err;
      void* fn = nt_cjit_get(dev, prog, err);
      return std::make_pair(fn, err);
    });
  }
  if (!wait && ctx->cjit_build.wait_for(std::chrono::seconds(0)) != std::future_status::ready) return false;
  auto r = ctx->cjit_build.get();
  ctx->cjit_fn = r.first;
  ctx->cjit_err = r.second;
  ctx->cjit_tried = true;
  return true;
}

// Default: batches of >= kCallJitMinReads reads take the specialised kernel
// once its background build (started by the first of them) is done -- until then,
// and for smaller batches, the ahead-of-time kernel (same results; no call
// ever waits for hiprtc).  NT_CALL_JIT=1: every batch, waiting for the build;
// NT_CALL_JIT=0: never.
static void* call_jit_fn(nt_ctx* ctx, uint64_t n_reads) {
  const int mode = call_jit_mode();
  if (mode == 0 || !ctx->jit || (mode < 0 && n_reads < kCallJitMinReads)) return nullptr;
  if (!cjit_collect(ctx, mode > 0)) return nullptr;
  return ctx->cjit_fn;
}

// a TVR of more than 32 letters: the calling kernel with wider neighbourhoods
static int long_tvr(const NtProgram& P) {
  for (int i = 0; i < P.n_tvr; ++i)
    if (P.tvr[i].m > 32) return 1;
  return 0;
}

// The calling of batch B (its list, or all its reads): the specialised
// kernel(s) when cfn, else the ahead-of-time kernel with np <= 2 ? 2 : 4
// lanes a read; at most 64 blocks a CU (grid-stride).
static hipError_t launch_call(nt_ctx* ctx, void* cfn, const NtBatch* B, const NtOut* O, const uint64_t* tm,
                              int fix_last, hipStream_t s) {
  const uint32_t* thr = (const uint32_t*)ctx->thr.p;
  const uint32_t ts = (uint32_t)ctx->thr_h.size();
  const int np = ctx->prog.n_pass;
  ++ctx->call_launches[cfn ? 1 : 0];
  // profiling: events around the calling kernel on its own stream (its span,
  // whether or not a scan runs beside it)
  hipEvent_t* ce = nullptr;
  if (ctx->profile && ctx->n_ev > 0 && ctx->cev_n[ctx->n_ev - 1] < nt_ctx::kMaxTsub + 2) {
    const int k = ctx->cev_n[ctx->n_ev - 1]++;
    ce = &ctx->cev[ctx->n_ev - 1][2 * k];
    (void)hipEventRecord(ce[0], s);
  }
  hipError_t e;
  if (cfn) {
    e = nt_cjit_launch(cfn, np, ctx->cu_count, s, ctx->prog_dev, B, O, tm, thr, ts, fix_last);
  } else {
    const uint64_t lanes = (B->list ? B->n_list : B->n_reads) * (np <= 2 ? 2u : 4u);
    const int grid = (int)std::max<uint64_t>(1, std::min<uint64_t>((lanes + 255) / 256, (uint64_t)ctx->cu_count * 64));
    e = nt_dev_launch_call(ctx->prog_dev, B, O, tm, thr, ts, fix_last, long_tvr(ctx->prog), grid, s);
  }
  if (ce) (void)hipEventRecord(ce[1], s);
  return e;
}

static int hip_fail(nt_ctx* ctx, hipError_t e, const char* what) {
  return fail(ctx, NT_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

extern "C" {

const char* nt_version(void) { return "nanotel-mi355x 0.1.0 (NanoTel v1.1.9-beta hot path)"; }

int nt_create(int device, nt_ctx** out) {
  if (!out) return NT_E_ARG;
  *out = nullptr;
  nt_ctx* ctx = new (std::nothrow) nt_ctx();
  if (!ctx) return NT_E_NOMEM;
  ctx->device = device;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    delete ctx;
    return NT_E_HIP;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    ctx->cu_count = prop.multiProcessorCount;
  e = hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete ctx;
    return NT_E_HIP;
  }
  ctx->stream = ctx->own_stream;
  e = hipMalloc(&ctx->prog_dev, sizeof(NtProgram));
  if (e != hipSuccess) {
    (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
    return NT_E_HIP;
  }
  *out = ctx;
  return NT_OK;
}

void nt_destroy(nt_ctx* ctx) {
  if (!ctx) return;
  // NT_DESTROY_TIMES=1 (diagnostics): the teardown's phases on stderr
  const bool tt = std::getenv("NT_DESTROY_TIMES") != nullptr;
  double t0 = now_s();
  auto lap = [&](const char* what) {
    if (!tt) return;
    const double t = now_s();
    std::fprintf(stderr, "nt_destroy: %s %.4f s\n", what, t - t0);
    t0 = t;
  };
  if (ctx->cjit_build.valid()) ctx->cjit_build.wait();
  lap("calling-kernel build");
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->call_stream) (void)hipStreamSynchronize(ctx->call_stream);
  lap("streams");
  if (ctx->prog_dev) (void)hipFree(ctx->prog_dev);
  if (ctx->ev_scan) (void)hipEventDestroy(ctx->ev_scan);
  if (ctx->ev_call) (void)hipEventDestroy(ctx->ev_call);
  for (hipEvent_t x : ctx->ev_done)
    if (x) (void)hipEventDestroy(x);
  if (ctx->call_stream) (void)hipStreamDestroy(ctx->call_stream);
  for (auto& a : ctx->ev)
    for (hipEvent_t ev : a) (void)hipEventDestroy(ev);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  lap("events and streams destroyed");
  delete ctx;
  lap("buffers freed");
}

const char* nt_last_error(const nt_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int nt_set_stream(nt_ctx* ctx, void* hip_stream) {
  if (!ctx) return NT_E_ARG;
  ctx->stream = hip_stream ? (hipStream_t)hip_stream : ctx->own_stream;
  return NT_OK;
}

// the context stream waits for everything on the calling stream (pipelined
// batches' last callings)
int nt_join(nt_ctx* ctx) {
  if (!ctx) return NT_E_ARG;
  if (!ctx->call_stream) return NT_OK;
  (void)hipSetDevice(ctx->device);
  hipError_t e;
  if ((e = hipEventRecord(ctx->ev_call, ctx->call_stream)) != hipSuccess ||
      (e = hipStreamWaitEvent(ctx->stream, ctx->ev_call, 0)) != hipSuccess)
    return hip_fail(ctx, e, "nt_join");
  return NT_OK;
}

int nt_wait_call(nt_ctx* ctx, uint32_t back) {
  if (!ctx) return NT_E_ARG;
  if (!ctx->pipelined || !ctx->ev_done[0] || back >= 2 || ctx->pipe_i < 1 + (uint64_t)back) return NT_OK;
  (void)hipSetDevice(ctx->device);
  // call c = pipe_i - 1 - back recorded ev_done[c & 1] after its last calling
  const hipError_t e = hipStreamWaitEvent(ctx->stream, ctx->ev_done[(ctx->pipe_i - 1 - back) & 1], 0);
  return e == hipSuccess ? NT_OK : hip_fail(ctx, e, "nt_wait_call");
}

int nt_set_pipelined(nt_ctx* ctx, int on) {
  if (!ctx) return NT_E_ARG;
  if (ctx->pipelined && !on) {
    const int rc = nt_join(ctx);
    if (rc) return rc;
  }
  ctx->pipelined = on != 0;
  return NT_OK;
}

int nt_synchronize(nt_ctx* ctx) {
  if (!ctx) return NT_E_ARG;
  const int rc = nt_join(ctx);
  if (rc) return rc;
  hipError_t e = hipStreamSynchronize(ctx->stream);
  return e == hipSuccess ? NT_OK : hip_fail(ctx, e, "hipStreamSynchronize");
}

int nt_compile(nt_ctx* ctx, const nt_params* prm, nt_program_info* info) {
  if (!ctx || !prm) return NT_E_ARG;
  NtProgram P;
  std::vector<uint32_t> thr;
  std::string err;
  const int rc = make_program(prm, P, thr, err);
  if (rc) return fail(ctx, rc, err);
  (void)hipSetDevice(ctx->device);
  hipError_t e = hipMemcpy(ctx->prog_dev, &P, sizeof P, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(ctx, e, "hipMemcpy(program)");
  if ((e = ctx->thr.ensure(thr.size() * 4)) != hipSuccess) return hip_fail(ctx, e, "hipMalloc(thr)");
  e = hipMemcpy(ctx->thr.p, thr.data(), thr.size() * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(ctx, e, "hipMemcpy(thr)");
  ctx->prog = P;
  ctx->thr_h = thr;
  ctx->params = *prm;
  ctx->compiled = true;
  ctx->jit = nt_jit_get(ctx->device, P, ctx->jit_fn, &ctx->tjit_fn, ctx->jit_err);
  if (ctx->cjit_build.valid()) ctx->cjit_build.wait();  // a previous program's build
  ctx->cjit_build = {};
  ctx->cjit_fn = nullptr;
  ctx->cjit_tried = false;
  ctx->tscan_bpc = 0;
  if (ctx->tjit_fn && std::getenv("NT_TSCAN") && std::getenv("NT_TSCAN")[0] == '0') ctx->tjit_fn = nullptr;
  if (ctx->tjit_fn) {
    ctx->tscan_bpc = nt_jit_blocks_per_cu(ctx->tjit_fn, 0);
    if (const char* v = std::getenv("NT_TSCAN_BPC"))  // tuning experiments: fewer resident blocks per CU
      ctx->tscan_bpc = std::min(ctx->tscan_bpc, std::atoi(v));
    if (ctx->tscan_bpc <= 0) ctx->tjit_fn = nullptr;
  }
  if (info) {
    info->n_pass = P.n_pass;
    info->n_pat = P.n_pat;
    info->n_tvr = P.n_tvr;
    info->n_hits = P.n_hits;
    info->raw_p1 = P.raw_p1;
    info->jit = ctx->jit ? 1 : 0;
    info->tscan = ctx->tjit_fn ? 1 : 0;
    info->count_bytes = ctx->prog.cnt8 ? 1 : 2;
  }
  return NT_OK;
}

// Read distribution of the scan (scan_reads): the 8 per-XCD queues, ~64 kb
// per claim and >= ~8 claims per wave.  NT_STATIC_FRAC (a static share
// before the queues, measured slower) and NT_CLAIM override (tuning).
struct QueuePlan {
  uint32_t claim, nstatic;
};
static QueuePlan queue_plan(uint64_t n_reads, uint64_t mean_len, uint64_t waves) {
  waves = std::max<uint64_t>(waves, 1);
  double frac = 0.0;
  if (const char* v = std::getenv("NT_STATIC_FRAC")) frac = std::min(1.0, std::max(0.0, std::atof(v)));
  const uint64_t nst = (uint64_t)(frac * (double)(n_reads / waves));
  const uint64_t dyn = n_reads - nst * waves;
  uint64_t c = (64000 + std::max<uint64_t>(mean_len, 1) / 2) / std::max<uint64_t>(mean_len, 1);
  c = std::min<uint64_t>(c, dyn / (8 * waves));
  if (const char* v = std::getenv("NT_CLAIM")) c = (uint64_t)std::max(1, std::atoi(v));
  return {(uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(c, 64)), (uint32_t)nst};
}

int nt_scan_call(nt_ctx* ctx, const nt_batch* batch, const nt_out* out, uint64_t max_len) {
  if (!ctx || !batch || !out) return NT_E_ARG;
  if (!ctx->compiled) return fail(ctx, NT_E_STATE, "nt_compile() not called");
  if (batch->n_reads == 0) return NT_OK;
  if (!out->win_counts || !out->start || !out->end || !out->density || !out->flags)
    return fail(ctx, NT_E_ARG, "win_counts/start/end/density/flags outputs are required");
  if (max_len > (1ull << 30)) return fail(ctx, NT_E_LIMIT, "read longer than 2^30 bases");
  // win_off / n_windows count PADDED rows (multiples of 64, nt_window_rows):
  // the aux scratch is sized from n_windows and indexed by the padded win_off
  if (batch->n_windows % 64)
    return fail(ctx, NT_E_ARG, "n_windows must be the sum of the padded window rows (a multiple of 64)");
  (void)hipSetDevice(ctx->device);
  const NtProgram& P = ctx->prog;
  const int np = P.n_pass, L = P.L, nh = P.n_hits;
  const int single = (P.n_pat == 1 && P.n_tvr == 0 && np == 2) ? 1 : 0;
  const int one = (single && P.pat[0].onehot) ? 1 : 0;
  const int m6 = (single && P.pat[0].m == 6) ? 1 : 0;
  // the bundle scan takes the bundled reads when the program has one and no
  // hit counters are asked for (a parity/debug output of the per-read scan)
  const bool tscan = ctx->tjit_fn && batch->bnd_read && batch->n_bundles && !out->hits;
  // the bundle scan stores 8 window counts at once: padded rows (nt_common.h) from a 16-byte aligned base
  if (tscan && (reinterpret_cast<uintptr_t>(out->win_counts) & 15))
    return fail(ctx, NT_E_ARG, "win_counts must be 16-byte aligned for the bundle scan");
  NtBatch B{batch->planes, batch->blk_off, batch->len, batch->win_off,
            batch->exc_off, batch->exc_pos, batch->exc_code, batch->n_reads,
            tscan ? batch->list : nullptr, tscan ? batch->n_list : 0,
            batch->bnd_read, tscan ? batch->n_bundles : 0};
  if (tscan && batch->n_list && !batch->list) return fail(ctx, NT_E_ARG, "n_list > 0 without a list");
  const uint64_t n_scan = tscan ? batch->n_list : batch->n_reads;  // reads of the per-read scan
  NtOut O{out->win_counts, out->start, out->end, out->density, out->flags, out->hits};
  hipError_t e;
  if (!ctx->lds_limit_set) {
    if ((e = nt_dev_set_lds_limit(kLdsCapBytes)) != hipSuccess) return hip_fail(ctx, e, "hipFuncSetAttribute");
    ctx->lds_limit_set = true;
  }
  const uint64_t tmw = nt_dev_tmask_words(batch->n_windows, batch->n_reads, np);
  // pipelined: the odd calls use the second aux buffer (the previous call's
  // calling may still read the other one)
  DevBuf& tmb = (ctx->pipelined && (ctx->pipe_i & 1)) ? ctx->tmask_alt : ctx->tmask;
  if ((e = tmb.ensure(tmw * 8)) != hipSuccess) return hip_fail(ctx, e, "hipMalloc(tmask)");
  uint64_t* tmask = (uint64_t*)tmb.p;
  // debugging: NT_DBG_POISON_AUX=<byte> fills the aux buffer first (every word read must be written)
  if (const char* v = std::getenv("NT_DBG_POISON_AUX"))
    (void)hipMemsetAsync(tmask, std::atoi(v) & 255, tmw * 8, ctx->stream);
  // per-wave window counters live in LDS up to the cap, in global scratch beyond
  const uint32_t max_nw = (uint32_t)window_count((int64_t)max_len, L);
  const int noslots = (single || ctx->jit) ? 1 : 0;  // register hit counters
  auto wg_bytes = [&](uint32_t nwc) { return (uint64_t)nt_dev_wave_words(noslots, nh, np, nwc) * 4u * 4u; };
  uint32_t cap_nw = max_nw;
  uint64_t len_cap = max_len;
  // the ahead-of-time scan keeps n_hits x 64 hit counters per wave in LDS:
  // from ~32 patterns on not even a read of no window fits the workgroup's
  // LDS, and every read takes the global-scratch instantiation
  const bool lds_fits = wg_bytes(0) <= kLdsCapBytes;
  if (!lds_fits) {
    cap_nw = 0;
    len_cap = 0;
  } else if (wg_bytes(max_nw) > kLdsCapBytes) {
    uint32_t lo = 0, hi = max_nw;
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) / 2;
      if (wg_bytes(mid) <= kLdsCapBytes) lo = mid; else hi = mid - 1;
    }
    cap_nw = lo;
    uint64_t a = 0, b = max_len;  // longest read with at most cap_nw windows
    while (a < b) {
      const uint64_t mid = (a + b + 1) / 2;
      if ((uint64_t)window_count((int64_t)mid, L) <= cap_nw) a = mid; else b = mid - 1;
    }
    len_cap = a;
  }
  const bool two = len_cap < max_len;
  // Sub-batches: the calling kernel of sub-batch k runs on a second stream
  // while the scan of sub-batch k+1 runs (NT_SUBBATCH, default 1 = serial);
  // NT_SCAN_WAVES caps the scan's blocks per CU to leave room for it.
  uint64_t nsub = 1;
  if (const char* v = std::getenv("NT_SUBBATCH")) nsub = std::max<uint64_t>(1, std::strtoull(v, nullptr, 10));
  nsub = std::min<uint64_t>(nsub, std::max<uint64_t>(1, batch->n_reads / 256));
  // the bundle scan's sub-batches (bundle ranges): the calling kernel of range
  // k runs on the call stream beside the bundle scan of range k+1 (the scan is
  // bandwidth-bound, the calling latency-bound), so only the last range's
  // calling is exposed.  Ranges of at most NT_TSUB_BUNDLES bundles (default
  // 16384 = 524,288 reads), at least 2, at most kMaxTsub; NT_TSUB sets the
  // count (1M x 50 kb, one box, two runs each: 3.43-3.45 ms per batch at 1,
  // 3.30-3.33 at 2, 3.38-3.41 at 3 geometric ranges, ratio 0.3)
  uint64_t tsub = 1;
  if (tscan) {
    nsub = 1;
    // pipelined, the last range's calling is hidden behind the next batch's
    // scan anyway: fewer, larger ranges (fewer range tails; same box, c10k
    // +1.4 %, c4 +1.5 %, c3 10 M +0.6 %)
    uint64_t per = ctx->pipelined ? 32768 : 16384;
    if (const char* v = std::getenv("NT_TSUB_BUNDLES")) per = std::max<uint64_t>(1, std::strtoull(v, nullptr, 10));
    tsub = std::max<uint64_t>(2, (batch->n_bundles + per - 1) / per);
    if (const char* v = std::getenv("NT_TSUB")) tsub = std::max<uint64_t>(1, std::strtoull(v, nullptr, 10));
    tsub = std::min<uint64_t>({tsub, std::max<uint64_t>(1, batch->n_bundles / 64), (uint64_t)nt_ctx::kMaxTsub});
  }
  int bpc_cap = 0;
  if (const char* v = std::getenv("NT_SCAN_WAVES")) bpc_cap = std::atoi(v);
  const bool piped = ctx->pipelined && (nsub > 1 || tsub > 1 || tscan);
  if ((nsub > 1 || tsub > 1 || piped) && !ctx->call_stream) {
    int prio = 0;  // NT_CALL_PRIO (tuning): the calling stream's priority, clamped to the device's range
    if (const char* v = std::getenv("NT_CALL_PRIO")) {
      int lo = 0, hi = 0;
      (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
      prio = std::max(std::min(std::atoi(v), std::max(lo, hi)), std::min(lo, hi));
    }
    if ((e = hipStreamCreateWithPriority(&ctx->call_stream, hipStreamNonBlocking, prio)) != hipSuccess)
      return hip_fail(ctx, e, "hipStreamCreate(call)");
    if ((e = hipEventCreateWithFlags(&ctx->ev_scan, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&ctx->ev_call, hipEventDisableTiming)) != hipSuccess)
      return hip_fail(ctx, e, "hipEventCreate");
    for (hipEvent_t& x : ctx->ev_done) {
      if ((e = hipEventCreateWithFlags(&x, hipEventDisableTiming)) != hipSuccess ||
          (e = hipEventRecord(x, ctx->call_stream)) != hipSuccess)
        return hip_fail(ctx, e, "hipEventCreate");
    }
  }
  // pipelined: this call's scans overwrite the aux buffer that the calling of
  // call pipe_i - 2 read
  if (ctx->pipelined && ctx->ev_done[0] &&
      (e = hipStreamWaitEvent(ctx->stream, ctx->ev_done[ctx->pipe_i & 1], 0)) != hipSuccess)
    return hip_fail(ctx, e, "stream dependency");
  // read queues: two per sub-batch (LDS and global-scratch launches) and one
  // per bundle range, zeroed on the stream
  const uint64_t nqueue = 2 * nsub + tsub;
  if ((e = ctx->queue.ensure(nqueue * NT_QUEUE_WORDS * 8)) != hipSuccess) return hip_fail(ctx, e, "hipMalloc(queue)");
  unsigned long long* queue = (unsigned long long*)ctx->queue.p;
  void* cfn = call_jit_fn(ctx, batch->n_reads);  // (built here on first use, before any timing event)
  ctx->cjit_last = cfn ? 1 : 0;
  hipEvent_t* ev = nullptr;
  if (ctx->profile) {
    if (ctx->n_ev == ctx->ev.size()) {
      std::array<hipEvent_t, 3 + 2 * (nt_ctx::kMaxTsub + 1)> a{};
      for (hipEvent_t& x : a)
        if ((e = hipEventCreate(&x)) != hipSuccess) return hip_fail(ctx, e, "hipEventCreate");
      std::array<hipEvent_t, 2 * (nt_ctx::kMaxTsub + 2)> c{};
      for (hipEvent_t& x : c)
        if ((e = hipEventCreate(&x)) != hipSuccess) return hip_fail(ctx, e, "hipEventCreate");
      ctx->ev.push_back(a);
      ctx->ev_nt.push_back(0);
      ctx->cev.push_back(c);
      ctx->cev_n.push_back(0);
    }
    ev = ctx->ev[ctx->n_ev++].data();
    ctx->ev_nt[ctx->n_ev - 1] = 0;
    ctx->cev_n[ctx->n_ev - 1] = 0;
    (void)hipEventRecord(ev[0], ctx->stream);
  }
  if ((e = hipMemsetAsync(queue, 0, nqueue * NT_QUEUE_WORDS * 8, ctx->stream)) != hipSuccess) return hip_fail(ctx, e, "hipMemsetAsync(queue)");
  if (tscan) {
    // the bundle scan first: one wave per bundle, exactly the resident blocks
    // (one per CU while a calling kernel runs beside it: room for its waves)
    const uint32_t thr_full = ctx->thr_h[std::min<size_t>((size_t)L, ctx->thr_h.size() - 1)];
    int tbpc = tsub > 1 ? 1 : ctx->tscan_bpc;
    if (const char* v = std::getenv("NT_TSCAN_RANGE_BPC"))  // tuning: blocks per CU beside the calling
      if (tsub > 1) tbpc = std::max(1, std::min(ctx->tscan_bpc, std::atoi(v)));
    // range sizes: geometric with NT_TRATIO (default 1 = equal).  Smaller later
    // ranges leave less calling exposed at the end but measured no better: the
    // calling beside a range's scan slows that scan (contention), 3.34-3.61 ms
    // at 3 ranges, ratio 0.25
    double ratio = 1.0;
    if (const char* v = std::getenv("NT_TRATIO")) ratio = std::atof(v);
    if (!(ratio > 0.0 && ratio <= 1.0)) ratio = 1.0;
    std::vector<uint64_t> bb(tsub + 1, 0);
    {
      double tot = 0.0, acc = 0.0, wk = 1.0;
      for (uint64_t k = 0; k < tsub; ++k, wk *= ratio) tot += wk;
      wk = 1.0;
      for (uint64_t k = 0; k < tsub; ++k, wk *= ratio) {
        acc += wk;
        bb[k + 1] = k + 1 == tsub ? batch->n_bundles
                                  : std::min<uint64_t>(batch->n_bundles, (uint64_t)(batch->n_bundles * (acc / tot)));
        bb[k + 1] = std::max(bb[k + 1], bb[k]);
      }
    }
    for (uint64_t k = 0; k < tsub; ++k) {
      const uint64_t b0 = bb[k], b1 = bb[k + 1];
      if (b1 == b0) continue;
      NtBatch Bt = B;  // bundles [b0, b1)
      Bt.bnd_read += NT_BUNDLE * b0;
      Bt.n_bundles = b1 - b0;
      const uint64_t wpb = (uint64_t)std::max(1, nt_jit_block_threads(ctx->tjit_fn) / 64);  // a wave per bundle
      const uint64_t tgrid = std::max<uint64_t>(1, std::min<uint64_t>((Bt.n_bundles + wpb - 1) / wpb, (uint64_t)ctx->cu_count * tbpc));
      const int pe = ev ? ctx->ev_nt[ctx->n_ev - 1] : 0;  // event pair of this launch
      if (ev) (void)hipEventRecord(ev[3 + 2 * pe], ctx->stream);
      e = nt_tjit_launch(ctx->tjit_fn, (int)tgrid, ctx->stream, &Bt, &O, tmask,
                         queue + (2 * nsub + k) * NT_QUEUE_WORDS, thr_full);
      if (e != hipSuccess) return hip_fail(ctx, e, "launch nt_tscan_jit");
      if (ev) {
        (void)hipEventRecord(ev[4 + 2 * pe], ctx->stream);
        ctx->ev_nt[ctx->n_ev - 1] = pe + 1;
      }
      // its reads' calling (the bundles' slots; the last window of each recounted)
      NtBatch Bc = B;
      Bc.list = Bt.bnd_read;
      Bc.n_list = NT_BUNDLE * Bt.n_bundles;
      hipStream_t cs = ctx->stream;
      if (tsub > 1 || piped) {
        if ((e = hipEventRecord(ctx->ev_scan, ctx->stream)) != hipSuccess ||
            (e = hipStreamWaitEvent(ctx->call_stream, ctx->ev_scan, 0)) != hipSuccess)
          return hip_fail(ctx, e, "stream dependency");
        cs = ctx->call_stream;
      }
      if ((e = launch_call(ctx, cfn, &Bc, &O, tmask, 1, cs)) != hipSuccess)
        return hip_fail(ctx, e, "launch nt_call_kernel");
    }
  }
  const uint32_t ww_lds = nt_dev_wave_words(noslots, nh, np, cap_nw);
  const size_t lds_bytes = (size_t)ww_lds * 4u * 4u;
  // exactly the resident blocks (the waves take reads from a queue)
  void* jit_lds = ctx->jit_fn[O.hits ? 0 : 2];
  void* jit_gmem = ctx->jit_fn[O.hits ? 1 : 3];
  int bpc = ctx->jit ? nt_jit_blocks_per_cu(jit_lds, lds_bytes)
                     : nt_dev_scan_blocks_per_cu(single, one, m6, 1, lds_bytes);
  if (bpc <= 0) bpc = 1;
  if (bpc_cap > 0) bpc = std::min(bpc, bpc_cap);
  const uint32_t ww_g = nt_dev_wave_words(noslots, nh, np, max_nw);
  const uint64_t grid_g = std::max<uint64_t>(1, std::min<uint64_t>((batch->n_reads + 3) / 4, (uint64_t)ctx->cu_count * 2));
  if (two && (e = ctx->scratch.ensure(grid_g * 4 * (uint64_t)ww_g * 4)) != hipSuccess)
    return hip_fail(ctx, e, "hipMalloc(scratch)");
  for (uint64_t k = 0; k < nsub; ++k) {
    const uint64_t r0 = batch->n_reads * k / nsub, r1 = batch->n_reads * (k + 1) / nsub;
    const uint64_t nr = r1 - r0;
    // the sub-batch: pointers advanced by r0 (win_off / blk_off / exc_off stay absolute);
    // the telomeric-mask base is per batch-global read index (tm_base), so shift it too
    NtBatch Bk = B;
    Bk.blk_off += r0;
    Bk.len += r0;
    Bk.win_off += r0;
    if (Bk.exc_off) Bk.exc_off += r0;
    Bk.n_reads = nr;
    NtOut Ok = O;
    Ok.start += 3 * r0;
    Ok.end += 3 * r0;
    Ok.density += 3 * r0;
    Ok.flags += r0;
    if (Ok.hits) Ok.hits += (uint64_t)nh * r0;
    uint64_t* tmk = tmask + 16 * r0 * (uint64_t)np;  // aux_base(win_off, r, np) of the global read index
    unsigned long long* q = queue + 2 * NT_QUEUE_WORDS * k;
    const uint64_t ns = tscan ? n_scan : nr;  // queue positions of the per-read scan
    const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((ns + 3) / 4, (uint64_t)ctx->cu_count * bpc));
    const QueuePlan qp = queue_plan(std::max<uint64_t>(ns, 1), batch->n_windows * (uint64_t)L / batch->n_reads, grid * 4);
    const uint32_t claim = qp.claim, nstatic = qp.nstatic;
    // the per-read scan beside the bundle scan (its list reads): one more
    // timed launch of the scan kernels (nt_kernel_times)
    const int pe = (ev && tscan && n_scan > 0) ? ctx->ev_nt[ctx->n_ev - 1] : -1;
    if (pe >= 0) (void)hipEventRecord(ev[3 + 2 * pe], ctx->stream);
    if (n_scan == 0 || !lds_fits)
      e = hipSuccess;
    else if (ctx->jit)
      e = nt_jit_launch(jit_lds, (int)grid, lds_bytes, ctx->stream, ctx->prog_dev,
                        (const uint32_t*)ctx->thr.p, &Bk, &Ok, tmk, q, 0u, (uint32_t)len_cap, claim, nstatic, ww_lds,
                        nullptr);
    else
      e = nt_dev_launch(ctx->prog_dev, (const uint32_t*)ctx->thr.p, &Bk, &Ok, tmk, q, 0u, (uint32_t)len_cap, claim, nstatic,
                        single, one, m6, 1, ww_lds, nullptr, (int)grid, ctx->stream);
    if (e != hipSuccess) return hip_fail(ctx, e, "launch nt_scan_kernel<lds>");
    if (two && n_scan > 0) {
      if (ctx->jit)
        e = nt_jit_launch(jit_gmem, (int)grid_g, 0, ctx->stream, ctx->prog_dev, (const uint32_t*)ctx->thr.p,
                          &Bk, &Ok, tmk, q + NT_QUEUE_WORDS, (uint32_t)len_cap, 0xFFFFFFFFu, 1u, 0u, ww_g, (uint32_t*)ctx->scratch.p);
      else
        e = nt_dev_launch(ctx->prog_dev, (const uint32_t*)ctx->thr.p, &Bk, &Ok, tmk, q + NT_QUEUE_WORDS, (uint32_t)len_cap,
                          0xFFFFFFFFu, 1u, 0u, single, 0, 0, 0, ww_g, (uint32_t*)ctx->scratch.p, (int)grid_g,
                          ctx->stream);
      if (e != hipSuccess) return hip_fail(ctx, e, "launch nt_scan_kernel<global>");
    }
    if (pe >= 0) {
      (void)hipEventRecord(ev[4 + 2 * pe], ctx->stream);
      ctx->ev_nt[ctx->n_ev - 1] = pe + 1;
    }
    if (tscan) {
      // the reads of the per-read scan (the bundled ones are called above)
      if (n_scan > 0) e = launch_call(ctx, cfn, &Bk, &Ok, tmk, 0, ctx->stream);
    } else if (nsub == 1) {
      if (ev) (void)hipEventRecord(ev[1], ctx->stream);
      e = launch_call(ctx, cfn, &Bk, &Ok, tmk, 0, ctx->stream);
    } else {
      // calling kernel of this sub-batch on the call stream, after its scan
      if ((e = hipEventRecord(ctx->ev_scan, ctx->stream)) != hipSuccess ||
          (e = hipStreamWaitEvent(ctx->call_stream, ctx->ev_scan, 0)) != hipSuccess)
        return hip_fail(ctx, e, "stream dependency");
      e = launch_call(ctx, cfn, &Bk, &Ok, tmk, 0, ctx->call_stream);
    }
    if (e != hipSuccess) return hip_fail(ctx, e, "launch nt_call_kernel");
  }
  if (nsub > 1 || tsub > 1 || piped) {
    if (ev) (void)hipEventRecord(ev[1], ctx->stream);  // end of the last scan
    if (piped) {  // the last calling stays in flight (nt_join)
      if ((e = hipEventRecord(ctx->ev_done[ctx->pipe_i & 1], ctx->call_stream)) != hipSuccess)
        return hip_fail(ctx, e, "hipEventRecord");
    } else if ((e = hipEventRecord(ctx->ev_call, ctx->call_stream)) != hipSuccess ||
               (e = hipStreamWaitEvent(ctx->stream, ctx->ev_call, 0)) != hipSuccess) {
      return hip_fail(ctx, e, "stream join");
    }
  }
  if (ctx->pipelined) ++ctx->pipe_i;
  if (ev) (void)hipEventRecord(ev[2], ctx->stream);
  return NT_OK;
}

// has_exc[r] = 1 for the reads whose exceptions reach more than NT_EXC_WINDOWS
// windows before their last (they stay on the per-read scan); the others are
// left as they are.
static void exc_marks(const NtProgram& P, const uint32_t* len, const uint32_t* exc_off, const uint32_t* exc_pos,
                      uint64_t n_reads, uint8_t* has_exc) {
  parallel_for(n_reads, [&](uint64_t r) {
    const uint32_t e0 = exc_off[r], e1 = exc_off[r + 1];
    if (e1 == e0) return;
    const int nw = (int)window_count((int64_t)len[r], P.L);
    if (exc_windows(exc_pos + e0, e1 - e0, (int)len[r], P.L, nw, P.m_max, NT_EXC_WINDOWS, [](int) {}) >
        NT_EXC_WINDOWS)
      has_exc[r] = 1;
  });
}

// Bundles of the bundle scan: the eligible reads (no non-ACGT letter beyond
// NT_EXC_WINDOWS windows, the program covered by nt_tscan.h) sorted by length,
// longest first (ties in input order), 32 to a bundle.  The scan addresses a
// bundle's planes from its lowest read's with 32-bit offsets: with blk_off
// given, a bundle whose reads' planes span more than kBundleSpan bytes goes to
// the per-read scan whole (the host path's batches are far smaller).
static constexpr uint64_t kBundleSpan = 0x7FFFFFF0ull;  // nt_tscan.h kTsMaxSpan

int nt_bundle_plan(nt_ctx* ctx, const uint32_t* len, const uint64_t* blk_off, const uint8_t* has_exc,
                   uint64_t n_reads, uint32_t* bnd_read, uint64_t* n_bundles, uint32_t* list, uint64_t* n_list) {
  if (!ctx || !n_bundles || !n_list || (n_reads && (!len || !bnd_read || !list))) return NT_E_ARG;
  if (!ctx->compiled) return fail(ctx, NT_E_STATE, "nt_compile() not called");
  const bool ok = nt_tscan_eligible(ctx->prog);
  std::vector<uint32_t> in;
  in.reserve(n_reads);
  std::vector<uint8_t> out(n_reads, 0);  // reads left to the per-read scan
  for (uint64_t r = 0; r < n_reads; ++r) {
    if (ok && len[r] > 0 && !(has_exc && has_exc[r])) in.push_back((uint32_t)r);
    else out[r] = 1;
  }
  std::stable_sort(in.begin(), in.end(), [&](uint32_t a, uint32_t b) { return len[a] > len[b]; });
  const uint64_t ng = (in.size() + NT_BUNDLE - 1) / NT_BUNDLE;
  uint64_t nb = 0;
  for (uint64_t g = 0; g < ng; ++g) {
    const uint64_t i0 = g * NT_BUNDLE, i1 = std::min<uint64_t>(in.size(), i0 + NT_BUNDLE);
    if (blk_off) {  // the bundle's planes within kBundleSpan bytes
      uint64_t lo = ~0ull, hi = 0;
      for (uint64_t i = i0; i < i1; ++i) {
        lo = std::min(lo, blk_off[in[i]]);
        hi = std::max(hi, blk_off[in[i]] + read_blocks(len[in[i]]));
      }
      if ((hi - lo) * 8 > kBundleSpan) {
        for (uint64_t i = i0; i < i1; ++i) out[in[i]] = 1;
        continue;
      }
    }
    for (uint64_t s = 0; s < NT_BUNDLE; ++s)
      bnd_read[nb * NT_BUNDLE + s] = i0 + s < i1 ? in[i0 + s] : 0xFFFFFFFFu;
    ++nb;
  }
  uint64_t nl = 0;
  for (uint64_t r = 0; r < n_reads; ++r)
    if (out[r]) list[nl++] = (uint32_t)r;
  *n_bundles = nb;
  *n_list = nl;
  return NT_OK;
}

int nt_exc_marks(nt_ctx* ctx, const uint32_t* len, const uint32_t* exc_off, const uint32_t* exc_pos,
                 uint64_t n_reads, uint8_t* has_exc) {
  if (!ctx || (n_reads && (!len || !has_exc))) return NT_E_ARG;
  if (!ctx->compiled) return fail(ctx, NT_E_STATE, "nt_compile() not called");
  std::memset(has_exc, 0, n_reads);
  if (exc_off && n_reads) {
    if (!exc_pos && exc_off[n_reads] > exc_off[0]) return NT_E_ARG;
    exc_marks(ctx->prog, len, exc_off, exc_pos, n_reads, has_exc);
  }
  return NT_OK;
}

int nt_call_jit_state(const nt_ctx* ctx) { return ctx ? ctx->cjit_last : 0; }

int nt_jit_prebuild(const nt_params* params, const char* arch) {
  NtProgram P;
  std::vector<uint32_t> thr;
  std::string err;
  const int rc = make_program(params, P, thr, err);
  if (rc) return rc;
  return nt_jit_prebuild_program(P, arch ? arch : "gfx950");
}

int nt_call_jit_wait(nt_ctx* ctx) {
  if (!ctx) return NT_E_ARG;
  if (!ctx->compiled) return fail(ctx, NT_E_STATE, "nt_compile() not called");
  if (!ctx->jit || call_jit_mode() == 0) return 0;
  cjit_collect(ctx, true);
  return ctx->cjit_fn ? 1 : 0;
}

int64_t nt_kernel_launches(const nt_ctx* ctx) { return ctx ? ctx->last_launches : NT_E_ARG; }

int64_t nt_call_kernel_times(const nt_ctx* ctx, double* call_ms) {
  if (!ctx) return NT_E_ARG;
  if (call_ms) *call_ms = ctx->last_call_ms;
  return ctx->last_call_launches;
}

int nt_call_launch_counts(const nt_ctx* ctx, int64_t* out2) {
  if (!ctx || !out2) return NT_E_ARG;
  out2[0] = ctx->call_launches[0];
  out2[1] = ctx->call_launches[1];
  return NT_OK;
}

int nt_set_profiling(nt_ctx* ctx, int on) {
  if (!ctx) return NT_E_ARG;
  ctx->profile = on != 0;
  ctx->n_ev = 0;
  return NT_OK;
}

int64_t nt_kernel_times(nt_ctx* ctx, double* scan_ms, double* call_ms) {
  if (!ctx || !ctx->profile) return NT_E_STATE;
  double a = 0.0, b = 0.0;
  int64_t launches = 0;
  for (size_t i = 0; i < ctx->n_ev; ++i) {
    launches += ctx->ev_nt[i] > 0 ? ctx->ev_nt[i] : 1;
    hipEvent_t* ev = ctx->ev[i].data();
    hipError_t e = hipEventSynchronize(ev[2]);
    if (e != hipSuccess) return hip_fail(ctx, e, "hipEventSynchronize");
    float x = 0.f, y = 0.f;
    if (ctx->ev_nt[i] > 0) {  // bundle scan: its kernels' spans; the rest is calling not hidden behind them
      float t = 0.f;
      if ((e = hipEventElapsedTime(&t, ev[0], ev[2])) != hipSuccess) return hip_fail(ctx, e, "hipEventElapsedTime");
      for (int k = 0; k < ctx->ev_nt[i]; ++k) {
        float z = 0.f;
        if ((e = hipEventElapsedTime(&z, ev[3 + 2 * k], ev[4 + 2 * k])) != hipSuccess)
          return hip_fail(ctx, e, "hipEventElapsedTime");
        x += z;
      }
      y = t - x;
    } else {
      if ((e = hipEventElapsedTime(&x, ev[0], ev[1])) != hipSuccess) return hip_fail(ctx, e, "hipEventElapsedTime");
      if ((e = hipEventElapsedTime(&y, ev[1], ev[2])) != hipSuccess) return hip_fail(ctx, e, "hipEventElapsedTime");
    }
    a += x;
    b += y;
  }
  double cms = 0.0;
  int64_t cl = 0;
  for (size_t i = 0; i < ctx->n_ev; ++i) {
    for (int k = 0; k < ctx->cev_n[i]; ++k) {
      hipEvent_t* ce = &ctx->cev[i][2 * k];
      hipError_t e = hipEventSynchronize(ce[1]);
      float z = 0.f;
      if (e == hipSuccess) e = hipEventElapsedTime(&z, ce[0], ce[1]);
      if (e != hipSuccess) return hip_fail(ctx, e, "hipEventElapsedTime(call)");
      cms += z;
      ++cl;
    }
  }
  ctx->last_call_ms = cms;
  ctx->last_call_launches = cl;
  if (scan_ms) *scan_ms = a;
  if (call_ms) *call_ms = b;
  ctx->last_launches = launches;
  const int64_t n = (int64_t)ctx->n_ev;
  ctx->n_ev = 0;
  return n;
}

// Pack a host chunk (2-bit planes + exception lists, --rc fused) and upload
// it to the context's device buffers; B describes the device batch.
static int upload_reads(nt_ctx* ctx, const char* const* seqs, const uint64_t* lens, uint64_t n_reads,
                        nt_batch* B, uint64_t* max_len, bool want_bundles) {
  const int L = ctx->prog.L;
  if (n_reads && (!seqs || !lens)) return fail(ctx, NT_E_ARG, "null reads");
  (void)hipSetDevice(ctx->device);
  hipError_t e;
  // the staging is reused: a previous call that failed after its uploads may
  // still be reading it (calls end synchronised otherwise, so this is free)
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize");
  // the layout depends on the lengths only: blk_off | win_off | len straight
  // into pinned staging, then ONE pass over the letters packs the planes
  // (nt_pack_count + nt_pack_reads read them twice)
  double tp = now_s();
  auto lap = [&](int k) {
    const double t = now_s();
    ctx->host_t[k] += t - tp;
    tp = t;
  };
  const size_t meta_bytes = n_reads * (8 + 8 + 4);
  if ((e = ctx->h_meta.ensure(meta_bytes)) != hipSuccess) return hip_fail(ctx, e, "hipHostMalloc(meta)");
  uint64_t* h_blk = (uint64_t*)ctx->h_meta.p;
  uint64_t* h_win = h_blk + n_reads;
  uint32_t* h_len = (uint32_t*)(h_win + n_reads);
  uint64_t tb = 0, tw = 0, ml = 0;
  for (uint64_t r = 0; r < n_reads; ++r) {
    if (lens[r] > 0xFFFFFFFFull) return fail(ctx, NT_E_LIMIT, "read " + std::to_string(r) + " is longer than 2^32-1");
    h_blk[r] = tb;
    h_win[r] = tw;
    h_len[r] = (uint32_t)lens[r];
    tb += read_blocks(lens[r]);
    tw += NT_WIN_ROWS((uint64_t)window_count((int64_t)lens[r], L));
    ml = std::max(ml, lens[r]);
  }
  const size_t pw = 2 * tb + 2;
  if ((e = ctx->h_planes.ensure(pw * 4)) != hipSuccess) return hip_fail(ctx, e, "hipHostMalloc(planes)");
  uint32_t* hp = (uint32_t*)ctx->h_planes.p;
  hp[pw - 2] = hp[pw - 1] = 0u;
  const int rc_flag = ctx->params.rc;
  lap(0);
  std::vector<int64_t> cnt(n_reads);
  parallel_for(n_reads, [&](uint64_t r) {
    cnt[r] = pack_one((const unsigned char*)seqs[r], lens[r], rc_flag, hp + 2 * h_blk[r], nullptr, nullptr);
  });
  uint64_t te = 0;
  for (uint64_t r = 0; r < n_reads; ++r) {  // the first bad read in input order, as nt_pack_count
    if (lens[r] == 0)
      return fail(ctx, NT_E_EMPTY_READ, "read " + std::to_string(r) + " is empty (seq(1, 0, by=L) errors)");
    if (cnt[r] < 0)
      return fail(ctx, NT_E_LETTER, "read " + std::to_string(r) + " has a letter outside DNA_ALPHABET");
    te += (uint64_t)cnt[r];
  }
  // reads with IUPAC letters: their exception lists (a second, rare pass)
  std::vector<uint32_t> h_eoff(te ? n_reads + 1 : 0), h_epos(te);
  std::vector<uint8_t> h_ecode(te);
  if (te) {
    if (te > 0xFFFFFFFFull) return fail(ctx, NT_E_LIMIT, "more than 2^32-1 non-ACGT letters in one call");
    uint64_t acc = 0;
    for (uint64_t r = 0; r < n_reads; ++r) {
      h_eoff[r] = (uint32_t)acc;
      acc += (uint64_t)cnt[r];
    }
    h_eoff[n_reads] = (uint32_t)acc;
    parallel_for(n_reads, [&](uint64_t r) {
      if (cnt[r] > 0)
        pack_one((const unsigned char*)seqs[r], lens[r], rc_flag, hp + 2 * h_blk[r], h_epos.data() + h_eoff[r],
                 h_ecode.data() + h_eoff[r]);
    });
  }
  lap(1);
#define NT_UP_PTR(buf, ptr, bytes)                                                           \
  e = ctx->buf.ensure(bytes);                                                                \
  if (e != hipSuccess) return hip_fail(ctx, e, "hipMalloc(" #buf ")");                       \
  if ((bytes) > 0) {                                                                         \
    e = hipMemcpyAsync(ctx->buf.p, ptr, bytes, hipMemcpyHostToDevice, ctx->stream);          \
    if (e != hipSuccess) return hip_fail(ctx, e, "hipMemcpyAsync(" #buf ")");                \
  }
#define NT_UP(buf, vec) NT_UP_PTR(buf, vec.data(), vec.size() * sizeof(vec[0]))
  NT_UP_PTR(planes, hp, pw * 4);
  NT_UP_PTR(blk_off, h_blk, n_reads * 8);
  NT_UP_PTR(len, h_len, n_reads * 4);
  NT_UP_PTR(win_off, h_win, n_reads * 8);
  if (te) {
    NT_UP(exc_off, h_eoff);
    NT_UP(exc_pos, h_epos);
    NT_UP(exc_code, h_ecode);
    // the exception lists are pageable vectors: finish their copies before they go
    if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize");
  }
  // the batch's bundles (bundle scan): the plan, uploaded beside the planes
  // (the scan reads the reads from the planes themselves)
  uint64_t nb = 0, nl = 0;
  std::vector<uint32_t> h_bread, h_list;
  if (ctx->tjit_fn && want_bundles) {
    // reads with non-ACGT letters join the bundles unless their exceptions
    // reach more than NT_EXC_WINDOWS windows (nt_common.h)
    std::vector<uint8_t> hx(n_reads, 0);
    if (te) exc_marks(ctx->prog, h_len, h_eoff.data(), h_epos.data(), n_reads, hx.data());
    h_bread.resize((n_reads + NT_BUNDLE - 1) / NT_BUNDLE * NT_BUNDLE + NT_BUNDLE);
    h_list.resize(n_reads + 1);
    int rc = nt_bundle_plan(ctx, h_len, h_blk, hx.data(), n_reads, h_bread.data(), &nb, h_list.data(), &nl);
    if (rc) return rc;
    h_bread.resize(nb * NT_BUNDLE);
    h_list.resize(nl);
    lap(2);
  }
  if (nb) {
    NT_UP(bnd_read, h_bread);
    if (nl) { NT_UP(list, h_list); }
    // the vectors are pageable: finish their copies before they go
    if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize");
  }
#undef NT_UP
#undef NT_UP_PTR
  *B = nt_batch{(const uint32_t*)ctx->planes.p, (const uint64_t*)ctx->blk_off.p,
                (const uint32_t*)ctx->len.p, (const uint64_t*)ctx->win_off.p,
                te ? (const uint32_t*)ctx->exc_off.p : nullptr,
                te ? (const uint32_t*)ctx->exc_pos.p : nullptr,
                te ? (const uint8_t*)ctx->exc_code.p : nullptr, n_reads, tw,
                nb ? (const uint32_t*)ctx->bnd_read.p : nullptr, nb,
                nl && nb ? (const uint32_t*)ctx->list.p : nullptr, nb ? nl : 0};
  lap(3);
  *max_len = ml;
  return NT_OK;
}

// --use_filter threshold: the smallest covered count c of the 200-base edge
// sub-read with c / 200 >= min_density * 0.8 (fp64, as R evaluates
// filter_density(..., min_density = global_min_density*0.8), NanoTel.R:2143)
static uint32_t filter_threshold(double min_density) {
  const double thr = min_density * 0.8;
  for (uint32_t c = 0; c <= 200; ++c)
    if ((double)c / 200.0 >= thr) return c;
  return 201;
}

int nt_filter_call(nt_ctx* ctx, const nt_batch* batch, uint8_t* keep) {
  if (!ctx || !batch || (batch->n_reads && !keep)) return NT_E_ARG;
  if (!ctx->compiled) return fail(ctx, NT_E_STATE, "nt_compile() not called");
  if (batch->n_reads == 0) return NT_OK;
  (void)hipSetDevice(ctx->device);
  NtBatch B{batch->planes, batch->blk_off, batch->len, batch->win_off,
            batch->exc_off, batch->exc_pos, batch->exc_code, batch->n_reads,
            nullptr, 0, nullptr, 0};
  const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>((batch->n_reads + 255) / 256, (uint64_t)ctx->cu_count * 16));
  const hipError_t e = nt_dev_launch_filter(ctx->prog_dev, &B, keep, filter_threshold(ctx->prog.min_density),
                                            ctx->prog.right_edge, (int)grid, ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "launch nt_filter_kernel");
  return NT_OK;
}

int nt_filter_host(nt_ctx* ctx, const char* const* seqs, const uint64_t* lens, uint64_t n_reads,
                   uint8_t* keep) {
  if (!ctx || (n_reads && (!seqs || !lens || !keep))) return NT_E_ARG;
  if (!ctx->compiled) return fail(ctx, NT_E_STATE, "nt_compile() not called");
  if (n_reads == 0) return NT_OK;
  nt_batch B;
  uint64_t ml = 0;
  int rc = upload_reads(ctx, seqs, lens, n_reads, &B, &ml, false);
  if (rc) return rc;
  hipError_t e;
  if ((e = ctx->flags.ensure(n_reads)) != hipSuccess) return hip_fail(ctx, e, "hipMalloc(flags)");
  if ((rc = nt_filter_call(ctx, &B, (uint8_t*)ctx->flags.p))) return rc;
  if ((e = hipMemcpyAsync(keep, ctx->flags.p, n_reads, hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess)
    return hip_fail(ctx, e, "hipMemcpyAsync(keep)");
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize");
  return NT_OK;
}

int nt_analyze_host(nt_ctx* ctx, const char* const* seqs, const uint64_t* lens, uint64_t n_reads,
                    int32_t* start, int32_t* end, double* density, uint8_t* flags,
                    void* win_counts, uint32_t* hits) {
  if (!ctx) return NT_E_ARG;
  if (!ctx->compiled) return fail(ctx, NT_E_STATE, "nt_compile() not called");
  if (n_reads == 0) return NT_OK;
  const int np = ctx->prog.n_pass;
  nt_batch B;
  uint64_t ml = 0;
  // bundles only when the scan will use them (no hit counters requested)
  int rc = upload_reads(ctx, seqs, lens, n_reads, &B, &ml, hits == nullptr);
  if (rc) return rc;
  const uint64_t tw = B.n_windows;
  hipError_t e;
  const uint64_t nwc = tw * np, cb = ctx->prog.cnt8 ? 1 : 2;  // count entries, bytes per entry
  if ((e = ctx->wc.ensure(std::max<uint64_t>(1, nwc) * cb)) != hipSuccess) return hip_fail(ctx, e, "hipMalloc(wc)");
  if ((e = ctx->start.ensure(n_reads * 3 * 4)) != hipSuccess) return hip_fail(ctx, e, "hipMalloc(start)");
  if ((e = ctx->end.ensure(n_reads * 3 * 4)) != hipSuccess) return hip_fail(ctx, e, "hipMalloc(end)");
  if ((e = ctx->dens.ensure(n_reads * 3 * 8)) != hipSuccess) return hip_fail(ctx, e, "hipMalloc(dens)");
  if ((e = ctx->flags.ensure(n_reads)) != hipSuccess) return hip_fail(ctx, e, "hipMalloc(flags)");
  const uint64_t nh = (uint64_t)ctx->prog.n_hits * n_reads;
  if ((e = ctx->hits.ensure(std::max<uint64_t>(1, nh) * 4)) != hipSuccess) return hip_fail(ctx, e, "hipMalloc(hits)");
  nt_out O{ctx->wc.p, (int32_t*)ctx->start.p, (int32_t*)ctx->end.p,
           (double*)ctx->dens.p, (uint8_t*)ctx->flags.p, hits ? (uint32_t*)ctx->hits.p : nullptr};
  double t0 = now_s();
  rc = nt_scan_call(ctx, &B, &O, ml);
  if (rc) return rc;
  if (ctx->pipelined && (rc = nt_join(ctx)) != NT_OK) return rc;  // the rows are read back below
  std::vector<uint8_t> h_flags(n_reads);
#define NT_DOWN(dst, buf, bytes)                                                              \
  e = hipMemcpyAsync(dst, ctx->buf.p, bytes, hipMemcpyDeviceToHost, ctx->stream);            \
  if (e != hipSuccess) return hip_fail(ctx, e, "hipMemcpyAsync(" #buf ")");
  NT_DOWN(start, start, n_reads * 3 * 4);
  NT_DOWN(end, end, n_reads * 3 * 4);
  NT_DOWN(density, dens, n_reads * 3 * 8);
  NT_DOWN(h_flags.data(), flags, n_reads);
  if (win_counts && nwc) { NT_DOWN(win_counts, wc, nwc * cb); }
  if (hits && nh) { NT_DOWN(hits, hits, nh * 4); }
#undef NT_DOWN
  e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) return hip_fail(ctx, e, "hipStreamSynchronize");
  const double t1 = now_s();
  ctx->host_t[4] += t1 - t0;
  if (flags) std::memcpy(flags, h_flags.data(), n_reads);
  for (uint64_t r = 0; r < n_reads; ++r) {
    const uint8_t f = h_flags[r];
    if (!(f & NT_FLAG_DONE)) return fail(ctx, NT_E_HIP, "read " + std::to_string(r) + " not processed");
    if (f & NT_FLAG_ERR_ALIGN)
      return fail(ctx, NT_E_ARG, "read " + std::to_string(r) +
                                     ": layout error (an odd blk_off, or its bundle's planes more than 2 GiB apart)");
    if (f & NT_FLAG_ERR_RIGHT)
      return fail(ctx, NT_E_RIGHT_EMPTY,
                  "read " + std::to_string(r) + ": find_right_telo on a read without windows");
    if (f & NT_FLAG_ERR_WIDTH)
      return fail(ctx, NT_E_NEG_WIDTH, "read " + std::to_string(r) + ": negative IRanges width");
  }
  ctx->host_t[5] += now_s() - t1;
  return NT_OK;
}

int nt_host_times(const nt_ctx* ctx, double* t6) {
  if (!ctx || !t6) return NT_E_ARG;
  for (int i = 0; i < 6; ++i) t6[i] = ctx->host_t[i];
  return NT_OK;
}

int nt_synth_device(nt_ctx* ctx, const nt_synth_params* sp, uint64_t n_reads, uint32_t* planes_dev) {
  if (!ctx || !sp || (!planes_dev && n_reads)) return NT_E_ARG;
  if (sp->read_len == 0) return fail(ctx, NT_E_ARG, "read_len must be > 0");
  (void)hipSetDevice(ctx->device);
  const NtSynth S = to_synth(sp);
  hipError_t e = nt_dev_launch_synth(&S, planes_dev, n_reads, ctx->stream);
  return e == hipSuccess ? NT_OK : hip_fail(ctx, e, "launch nt_synth_kernel");
}

int nt_rc_device(nt_ctx* ctx, const uint32_t* planes_in, uint32_t* planes_out, const uint64_t* blk_off_dev,
                 const uint32_t* len_dev, uint64_t n_reads) {
  if (!ctx || (n_reads && (!planes_in || !planes_out || !blk_off_dev || !len_dev))) return NT_E_ARG;
  if (planes_in == planes_out && n_reads) return fail(ctx, NT_E_ARG, "nt_rc_device is out of place");
  (void)hipSetDevice(ctx->device);
  const hipError_t e = nt_dev_launch_rc(planes_in, planes_out, blk_off_dev, len_dev, n_reads, ctx->cu_count, ctx->stream);
  return e == hipSuccess ? NT_OK : hip_fail(ctx, e, "launch nt_rc_kernel");
}

int nt_uniform_layout_device(nt_ctx* ctx, uint64_t n_reads, uint64_t read_len, int32_t subseq_length,
                             uint64_t* blk_off_dev, uint32_t* len_dev, uint64_t* win_off_dev) {
  if (!ctx || read_len == 0 || read_len > 0xFFFFFFFFull) return NT_E_ARG;
  (void)hipSetDevice(ctx->device);
  const uint64_t nblk = read_blocks(read_len);
  const uint64_t nw = NT_WIN_ROWS((uint64_t)window_count((int64_t)read_len, subseq_length));  // padded rows
  hipError_t e = nt_dev_launch_uniform_layout(n_reads, nblk, read_len, nw, blk_off_dev, len_dev,
                                              win_off_dev, ctx->stream);
  return e == hipSuccess ? NT_OK : hip_fail(ctx, e, "launch nt_layout_kernel");
}

}  // extern "C"
