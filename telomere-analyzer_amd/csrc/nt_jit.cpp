// nt_jit.cpp -- run-time specialisation of the scan kernel (hiprtc).
//
// nt_compile() knows the pattern set; the scan's inner loop is dominated by
// the per-letter tests, so the scan is recompiled for it: every letter
// becomes a compile-time truth table over the 2-bit base (one v_bitop3 per
// DISTINCT letter test per word, shared across letters and patterns), the
// pattern lengths become compile-time (unrolled, 3-letter majority combine),
// and the hit counters live in registers.  The source is nt_scan.h itself
// (embedded at build time, nt_jit_src.inc) plus a generated pattern-set type.
// Code objects are cached per (device, source) for the life of the process.
// If hiprtc is unavailable the ahead-of-time kernels serve (NT_JIT=0 forces
// that); nt_program_info.jit reports which one runs.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>
#include <utime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "nt_common.h"

extern "C" hipError_t nt_dev_launch_combine(const NtBatch* B, const NtOut* O, int np, int grid, hipStream_t stream);

namespace {

#include "nt_jit_src.inc"  // kJitCommon, kJitDevice, kJitScan (raw string literals)

struct JitEntry {
  hipModule_t mod = nullptr;
  hipFunction_t fn[4] = {};  // [no hits ? 2 : 0] + [global scratch ? 1 : 0]
  hipFunction_t tfn = nullptr;  // the bundle scan (nt_tscan.h), when the program has one
  std::string err;
};

std::mutex g_mu;
std::map<std::string, JitEntry> g_cache;

// the calling kernel's modules (a separate hiprtc program: ~20 s to build, so
// it is built only for batches that pay for it, see nt_host.cpp)
// fn[0]: the one-kernel form (Call::run); split: fn[p] = pass p's kernel
// (Call<CS, p>::run_pass), then nt_call_combine_kernel.
struct CallEntry {
  hipModule_t mod = nullptr;
  hipFunction_t fn[3] = {};
  int nfn = 0;
  bool split = false;
  std::string err;
};
std::map<std::string, CallEntry> g_ccache;

// NT_JIT_OPTS (extra hiprtc options, e.g. -D switches of timing experiments)
// is honoured only by a tuning build of the library (make EXTRA=-DNT_TUNING_BUILD):
// the product library compiles every kernel as shipped, whatever the
// environment says.
const char* jit_opts() {
#ifdef NT_TUNING_BUILD
  return std::getenv("NT_JIT_OPTS");
#else
  return nullptr;
#endif
}

// eq: the code-equality truth tables (fixed=TRUE, the edge steps) instead of the scan's
std::string pat_type(const NtPat& P, bool eq = false) {
  std::string s = "nt::CtPat<" + std::to_string(P.m);
  for (int j = 0; j < P.m; ++j) s += ", " + std::to_string((int)(eq ? P.tt_eq[j] : P.tt_scan[j]));
  return s + ">";
}

const char* const kTypedefs =
    "typedef __hip_internal::uint8_t uint8_t;\n"
    "typedef __hip_internal::uint16_t uint16_t;\n"
    "typedef __hip_internal::uint32_t uint32_t;\n"
    "typedef __hip_internal::uint64_t uint64_t;\n"
    "typedef __hip_internal::int32_t int32_t;\n"
    "typedef __hip_internal::int64_t int64_t;\n";

}  // namespace

// The bundle scan (nt_tscan.h) covers programs whose patterns are at least 2
// letters long, in at most kTsMaxGroups (4) distinct lengths per list (one
// walk group per length; mixed-length lists such as "TTAGGG TTAGG"), with
// subseq_length L <= 170 (8-bit window counts of the transposed output) and
// 2 (max m - 1) < L (the read's last window, recounted by the calling kernel,
// holds every position whose letters reach past the read end), and patterns /
// TVRs of at most 32 letters (the walk's history registers grow with the
// longest).  Others take the per-read scan only.
bool nt_tscan_eligible(const NtProgram& P) {
  if (P.n_pat < 1 || P.L > 170) return false;
  auto lengths = [](const NtPat* v, int n, int& mn, int& mx) {
    bool seen[65] = {};
    int d = 0;
    for (int i = 0; i < n; ++i) {
      const int m = v[i].m;
      mn = m < mn ? m : mn;
      mx = m > mx ? m : mx;
      if (m >= 1 && m <= 64 && !seen[m]) {
        seen[m] = true;
        ++d;
      }
    }
    return d;
  };
  int mn = 1 << 30, M = 0;
  const int dp = lengths(P.pat, P.n_pat, mn, M);
  const int dt = lengths(P.tvr, P.n_tvr, mn, M);
  return mn >= 2 && dp <= 4 && dt <= 4 && M <= 32 && 2 * (M - 1) < P.L;
}

namespace {

// The bundle scan's pattern list with the patterns of one length that differ
// in a single letter merged into one (that letter's truth table the union):
// TTAGGG + TCAGGG -> TYAGGG.  The walk counts coverage only, and for two
// patterns P, Q equal but at letter k the <= 1-mismatch matches of P or Q are
// exactly those of the merged R (x_k in P's or Q's set: R's mismatches are P's
// or Q's; x_k in neither: R's one mismatch is at k and P's is too), as are the
// exact ones -- one combine a step instead of two (c4's TTAGGG TCAGGG).  The
// per-read scan keeps the list as given (its hit counters are per pattern).
std::string merged_types(const NtPat* v, int n) {
  struct T {
    int m;
    std::vector<int> tt;
  };
  std::vector<T> ps;
  for (int i = 0; i < n; ++i) {
    T t{v[i].m, std::vector<int>(v[i].tt_scan, v[i].tt_scan + v[i].m)};
    bool dup = false;
    for (const T& q : ps) dup = dup || (q.m == t.m && q.tt == t.tt);
    if (!dup) ps.push_back(t);
  }
  for (bool again = true; again;) {
    again = false;
    for (size_t i = 0; i < ps.size() && !again; ++i)
      for (size_t j = i + 1; j < ps.size() && !again; ++j) {
        if (ps[i].m != ps[j].m) continue;
        int k = -1, nd = 0;
        for (int x = 0; x < ps[i].m; ++x)
          if (ps[i].tt[x] != ps[j].tt[x]) {
            k = x;
            ++nd;
          }
        if (nd != 1) continue;
        ps[i].tt[k] |= ps[j].tt[k];
        ps.erase(ps.begin() + (long)j);
        again = true;
      }
  }
  std::string out;
  for (size_t i = 0; i < ps.size(); ++i) {
    out += (i ? ", " : "") + std::string("nt::CtPat<") + std::to_string(ps[i].m);
    for (int t : ps[i].tt) out += ", " + std::to_string(t);
    out += ">";
  }
  return out;
}

std::string jit_source(const NtProgram& P) {
  std::string pats, tvrs;
  for (int i = 0; i < P.n_pat; ++i) pats += (i ? ", " : "") + pat_type(P.pat[i]);
  for (int i = 0; i < P.n_tvr; ++i) tvrs += (i ? ", " : "") + pat_type(P.tvr[i]);
  const std::string tpats = merged_types(P.pat, P.n_pat), ttvrs = merged_types(P.tvr, P.n_tvr);
  std::string s = kTypedefs;
  s += "#include \"nt_tscan.h\"\n";
  s += "using JitSet = nt::CtSet<nt::CtList<" + pats + ">, nt::CtList<" + tvrs + ">>;\n";
  if (nt_tscan_eligible(P)) {
    s += "using TPats = nt::CtList<" + tpats + ">;\nusing TTvrs = nt::CtList<" + ttvrs + ">;\n";
    s += "using TJit = nt::TProg<TPats, TTvrs, " + std::to_string(P.L) + ">;\n";
    // one wave per bundle; as many waves a workgroup (at most 4, one per
    // SIMD) as their LDS (slots, output rows, the half-stripe buffer) fits in
    // the CU's 160 KB; ~420 registers a lane: one wave per SIMD
    s += R"(
constexpr int kTsW = nt::ts_lds_words<TJit::kNP, TJit::kL>();
constexpr int kTsNW = 40960 / kTsW < 4 ? 40960 / kTsW : 4;
static_assert(kTsNW >= 1, "bundle-scan LDS");
extern "C" __global__ void __launch_bounds__(kTsNW * 64) __attribute__((amdgpu_waves_per_eu(1)))
nt_tscan_jit(NtBatch B, NtOut O, uint64_t* __restrict__ tmask, unsigned long long* __restrict__ queue,
             uint32_t thr_full) {
  __shared__ uint32_t tsl[kTsNW * kTsW];
  nt::tscan_bundles<TJit, TPats, TTvrs>(B, O, tmask, queue, thr_full, tsl + (threadIdx.x >> 6) * kTsW);
}
)";
  }
  s += R"(
#ifdef NT_SCAN_WAVES_EU
#define NT_SCAN_ATTR __attribute__((amdgpu_waves_per_eu(NT_SCAN_WAVES_EU)))
#else
#define NT_SCAN_ATTR
#endif
#define NT_JIT_KERNELS(NAME, HITS)                                                                     \
  extern "C" __global__ void __launch_bounds__(256) NT_SCAN_ATTR                                       \
  NAME##_lds(const NtProgram* __restrict__ prog, const uint32_t* __restrict__ thr, NtBatch B, NtOut O, \
             uint64_t* __restrict__ tmask, unsigned long long* __restrict__ queue, uint32_t len_lo,    \
             uint32_t len_hi, uint32_t claim, uint32_t nstatic, uint32_t wave_words,                   \
             uint32_t* __restrict__ gscr) {                                                           \
    extern __shared__ uint32_t smem[];                                                                 \
    nt::scan_reads<JitSet, true, HITS>(prog, thr, B, O, tmask, queue, len_lo, len_hi, claim, nstatic,  \
                                       smem + (threadIdx.x >> 6) * wave_words,                         \
                                       reinterpret_cast<nt::DbgRec*>(gscr));                           \
  }                                                                                                    \
  extern "C" __global__ void __launch_bounds__(256)                                                    \
  NAME##_gmem(const NtProgram* __restrict__ prog, const uint32_t* __restrict__ thr, NtBatch B, NtOut O,\
              uint64_t* __restrict__ tmask, unsigned long long* __restrict__ queue, uint32_t len_lo,   \
              uint32_t len_hi, uint32_t claim, uint32_t nstatic, uint32_t wave_words,                  \
              uint32_t* __restrict__ gscr) {                                                          \
    const uint64_t gw = (uint64_t)blockIdx.x * nt::kNWaves + (threadIdx.x >> 6);                       \
    nt::scan_reads<JitSet, false, HITS>(prog, thr, B, O, tmask, queue, len_lo, len_hi, claim, nstatic, \
                                        gscr + gw * wave_words);                                       \
  }
// with the matchPattern hit counters, and without (the caller passed no hits buffer)
NT_JIT_KERNELS(nt_scan_jit, true)
NT_JIT_KERNELS(nt_scan_jit_nh, false)
)";
  return s;
}

}  // namespace

// The per-pass split of the calling kernel: a kernel per pass, each with its
// pass's mismatch rule, TVR use and raw views compile-time and registers of
// its own (the P1 / P2 kernels hold no TVR code), and no idle lane (the
// one-kernel form gives a 3-pass read 4 lanes).  Default for 3-pass programs;
// NT_CALL_SPLIT=0 / 1 forces it off / on.
bool nt_call_split(const NtProgram& P) {
  const char* e = std::getenv("NT_CALL_SPLIT");
  if (e && *e) return e[0] == '1';
  return P.n_pass == 3;
}

namespace {

// The program's source of the calling kernel (nt_call.h) with its patterns as types.
std::string call_source(const NtProgram& P) {
  std::string pats, tvrs, pats_eq, tvrs_eq;
  for (int i = 0; i < P.n_pat; ++i) {
    pats += (i ? ", " : "") + pat_type(P.pat[i]);
    pats_eq += (i ? ", " : "") + pat_type(P.pat[i], true);
  }
  for (int i = 0; i < P.n_tvr; ++i) {
    tvrs += (i ? ", " : "") + pat_type(P.tvr[i]);
    tvrs_eq += (i ? ", " : "") + pat_type(P.tvr[i], true);
  }
  std::string s = kTypedefs;
  s += "#include \"nt_call.h\"\n";
  s += "using JitCall = nt::CtCall<nt::CtList<" + pats + ">, nt::CtList<" + tvrs + ">, nt::CtList<" + pats_eq +
       ">, nt::CtList<" + tvrs_eq + ">, " + (P.raw_p1 ? "true" : "false") + ">;\n";
  if (nt_call_split(P)) {
    // per-pass occupancy: NT_CALL_WAVES_P<p> (the spill fallback sets one to 2)
    for (int p = 0; p < P.n_pass; ++p) {
      const std::string ps = std::to_string(p);
      s += "#ifndef NT_CALL_WAVES_P" + ps + "\n#define NT_CALL_WAVES_P" + ps + " NT_CALL_WAVES_PER_EU\n#endif\n";
      s += "#undef NT_CALL_ATTR\n#define NT_CALL_ATTR __attribute__((amdgpu_waves_per_eu(NT_CALL_WAVES_P" + ps + ")))\n";
      s += "NT_CALL_KERNEL_PASS(nt_call_jit_p" + ps + ", JitCall, " + ps + ")\n";
    }
  } else {
    s += "NT_CALL_KERNEL(nt_call_jit, JitCall)\n";
  }
  return s;
}

// ---- on-disk code-object cache: a hiprtc build of the calling kernel takes
// 5-20 s (the scan's 1-3 s), once per pattern set; the code object is kept
// under $NT_JIT_CACHE (default $XDG_CACHE_HOME/nanotel or ~/.cache/nanotel),
// keyed by a hash of everything that determines it: the program source, the
// embedded headers (so a rebuilt library with changed kernels misses), the
// options, the target and the hiprtc version.  NT_JIT_CACHE=0 turns it off;
// an unwritable directory only means no cache.
uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
  const unsigned char* c = (const unsigned char*)p;
  for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
  return h;
}

// $NT_JIT_CACHE, else jitcache/ next to libnanotel.so (in-tree: it travels
// with the tree, and __graft_entry__.build() fills it for the benchmark's
// pattern sets), else ~/.cache/nanotel when that one is not writable
std::string cache_dir() {
  const char* v = std::getenv("NT_JIT_CACHE");
  if (v && std::strcmp(v, "0") == 0) return "";
  if (v && *v) return v;
  Dl_info di;
  if (dladdr((const void*)&fnv1a, &di) && di.dli_fname) {
    std::string d = di.dli_fname;
    const size_t k = d.rfind('/');
    d = (k == std::string::npos ? std::string(".") : d.substr(0, k)) + "/jitcache";
    (void)mkdir(d.c_str(), 0755);
    if (access(d.c_str(), W_OK | X_OK) == 0) return d;
  }
  const char* x = std::getenv("XDG_CACHE_HOME");
  if (x && *x) return std::string(x) + "/nanotel";
  const char* h = std::getenv("HOME");
  return h && *h ? std::string(h) + "/.cache/nanotel" : "";
}

bool cache_read(const std::string& path, std::vector<char>& code) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  bool ok = n > 0;
  if (ok) {
    code.resize((size_t)n);
    ok = std::fread(code.data(), 1, (size_t)n, f) == (size_t)n;
  }
  std::fclose(f);
  // a hit marks the object as in use (tools/jit_cache_gc.sh drops the objects
  // no prebuild touched)
  if (ok) (void)utime(path.c_str(), nullptr);
  return ok;
}

void cache_write(const std::string& dir, const std::string& path, const std::vector<char>& code) {
  std::string d;  // mkdir -p
  for (size_t i = 0; i <= dir.size(); ++i) {
    if (i == dir.size() || dir[i] == '/') {
      if (!d.empty()) (void)mkdir(d.c_str(), 0755);
    }
    if (i < dir.size()) d += dir[i];
  }
  const std::string tmp = path + ".tmp." + std::to_string((long)getpid()) + "." +
                          std::to_string((unsigned long long)(uintptr_t)&code);
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return;
  const bool ok = std::fwrite(code.data(), 1, code.size(), f) == code.size();
  if (std::fclose(f) == 0 && ok) (void)std::rename(tmp.c_str(), path.c_str());  // atomic publish
  else (void)std::remove(tmp.c_str());
}

// The code object of src for arch (--offload-arch=...): from the on-disk
// cache (unless fresh), else compiled by hiprtc (and cached).  The cache key
// hashes the source, the embedded headers and every compiler option (the
// fixed ones below included: -ffp-contract decides the fp64 densities'
// rounding), plus the hiprtc version.  *cpath_out: the cache file used.
bool get_code(const std::string& arch, const std::string& src, std::vector<char>& code, std::string& err,
              bool fresh = false, std::string* cpath_out = nullptr) {
  const char* hdrs[] = {kJitCommon, kJitDevice, kJitScan, kJitTScan, kJitCall};
  const char* names[] = {"nt_common.h", "nt_device.h", "nt_scan.h", "nt_tscan.h", "nt_call.h"};
  std::vector<std::string> extra;  // NT_JIT_OPTS: extra compiler options (tuning builds only)
  if (const char* v = jit_opts()) {
    std::string t;
    for (const char* p = v;; ++p) {
      if (*p == ' ' || *p == 0) {
        if (!t.empty()) extra.push_back(t);
        t.clear();
        if (*p == 0) break;
      } else {
        t += *p;
      }
    }
  }
  // max-ilp machine scheduling: scan 3.41 -> 3.37 ms at 1M x 50 kb (c4 -0.8 %, c10k
  // unchanged; tools/jit_sweep.sh); it orders the VALU stream with fewer slow/fast
  // alternations
  std::vector<const char*> opts = {arch.c_str(), "-O3", "-std=c++17", "-ffp-contract=off", "-mllvm",
                                   "-amdgpu-sched-strategy=max-ilp"};
  for (const std::string& x : extra) opts.push_back(x.c_str());
  const std::string dir = cache_dir();
  std::string cpath;
  if (!dir.empty()) {
    uint64_t h = 1469598103934665603ull;
    h = fnv1a(h, src.data(), src.size());
    // the headers the source reaches: nt_common / nt_device / nt_scan always,
    // nt_tscan.h and nt_call.h when it includes them (a bundle-scan change
    // leaves the calling kernels' objects valid, and the other way round)
    for (int i = 0; i < 5; ++i)
      if (i < 3 || src.find(std::string("#include \"") + names[i] + "\"") != std::string::npos)
        h = fnv1a(h, hdrs[i], std::strlen(hdrs[i]));
    for (const char* o : opts) h = fnv1a(h, o, std::strlen(o) + 1);  // NUL-separated
    int maj = 0, mnr = 0;
    (void)hiprtcVersion(&maj, &mnr);
    h = fnv1a(h, &maj, sizeof maj);
    h = fnv1a(h, &mnr, sizeof mnr);
    char hex[24];
    std::snprintf(hex, sizeof hex, "%016llx", (unsigned long long)h);
    cpath = dir + "/nt_" + hex + ".co";
    if (cpath_out) *cpath_out = cpath;
    if (!fresh && cache_read(cpath, code)) return true;
  }
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "nt_jit.hip", 5, hdrs, names) != HIPRTC_SUCCESS) {
    err = "hiprtcCreateProgram failed";
    return false;
  }
  const hiprtcResult rc = hiprtcCompileProgram(prog, (int)opts.size(), opts.data());
  if (rc != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n + 1, '\0');
    hiprtcGetProgramLog(prog, &log[0]);
    err = std::string("hiprtc: ") + hiprtcGetErrorString(rc) + "\n" + log.c_str();
    hiprtcDestroyProgram(&prog);
    return false;
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  code.resize(n);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  if (!cpath.empty()) cache_write(dir, cpath, code);
  return true;
}

std::string device_arch(int device) {
  hipDeviceProp_t prop;
  std::string arch = "--offload-arch=gfx950";
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
    std::string a = prop.gcnArchName;
    arch = "--offload-arch=" + a.substr(0, a.find(':'));
  }
  return arch;
}

// src as a loaded module on the calling thread's device
bool compile_module(int device, const std::string& src, hipModule_t& mod, std::string& err) {
  std::vector<char> code;
  std::string cpath;
  const std::string arch = device_arch(device);
  if (!get_code(arch, src, code, err, false, &cpath)) return false;
  hipError_t he = hipModuleLoadData(&mod, code.data());
  if (he != hipSuccess && !cpath.empty()) {
    // a cached object the runtime rejects (truncated, another runtime's):
    // dropped and compiled afresh, once
    (void)std::remove(cpath.c_str());
    if (!get_code(arch, src, code, err, true)) return false;
    he = hipModuleLoadData(&mod, code.data());
  }
  if (he != hipSuccess) {
    err = std::string("hipModuleLoadData: ") + hipGetErrorString(he);
    return false;
  }
  return true;
}

bool compile(int device, const std::string& src, JitEntry& e) {
  if (!compile_module(device, src, e.mod, e.err)) return false;
  hipError_t he = hipSuccess;
  const char* names4[4] = {"nt_scan_jit_lds", "nt_scan_jit_gmem", "nt_scan_jit_nh_lds", "nt_scan_jit_nh_gmem"};
  for (int i = 0; i < 4 && he == hipSuccess; ++i) he = hipModuleGetFunction(&e.fn[i], e.mod, names4[i]);
  if (he != hipSuccess) {
    e.err = std::string("hipModuleGetFunction: ") + hipGetErrorString(he);
    return false;
  }
  if (src.find("nt_tscan_jit(") != std::string::npos &&
      hipModuleGetFunction(&e.tfn, e.mod, "nt_tscan_jit") != hipSuccess)
    e.tfn = nullptr;
  return true;
}

}  // namespace

// Returns true with the four kernels of the program's pattern set (fn[i]:
// i = [no hit counters ? 2 : 0] + [global scratch ? 1 : 0]), false (and a
// message) when specialisation is off or failed.
bool nt_jit_get(int device, const NtProgram& P, void* fn[4], void** tfn, std::string& err) {
  if (tfn) *tfn = nullptr;
  const char* env = std::getenv("NT_JIT");
  if (env && env[0] == '0') {
    err = "NT_JIT=0";
    return false;
  }
  const std::string src = jit_source(P);
  const char* xo = jit_opts();
  const std::string key = std::to_string(device) + "\n" + (xo ? xo : "") + "\n" + src;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_cache.find(key);
  if (it == g_cache.end()) {
    JitEntry e;
    compile(device, src, e);
    it = g_cache.emplace(key, e).first;
  }
  if (!it->second.fn[3]) {
    err = it->second.err;
    return false;
  }
  for (int i = 0; i < 4; ++i) fn[i] = (void*)it->second.fn[i];
  if (tfn) *tfn = (void*)it->second.tfn;
  return true;
}

// a JIT kernel's block size (its __launch_bounds__: the bundle scan's is 64
// kTsNW, a wave per bundle and as many as the CU's LDS holds; 256 otherwise)
static int jit_threads(void* fn) {
  int v = 0;
  if (hipFuncGetAttribute(&v, HIP_FUNC_ATTRIBUTE_MAX_THREADS_PER_BLOCK, (hipFunction_t)fn) != hipSuccess || v <= 0)
    return 256;
  return v;
}

int nt_jit_block_threads(void* fn) { return jit_threads(fn); }

hipError_t nt_tjit_launch(void* fn, int grid, hipStream_t stream, const NtBatch* B, const NtOut* O,
                          uint64_t* tmask, unsigned long long* queue, uint32_t thr_full) {
  NtBatch b = *B;
  NtOut o = *O;
  void* args[] = {&b, &o, &tmask, &queue, &thr_full};
  return hipModuleLaunchKernel((hipFunction_t)fn, (unsigned)grid, 1, 1, (unsigned)jit_threads(fn), 1, 1, 0, stream,
                               args, nullptr);
}

hipError_t nt_jit_launch(void* fn, int grid, size_t lds_bytes, hipStream_t stream,
                         const NtProgram* prog, const uint32_t* thr, const NtBatch* B,
                         const NtOut* O, uint64_t* tmask, unsigned long long* queue,
                         uint32_t len_lo, uint32_t len_hi, uint32_t claim, uint32_t nstatic, uint32_t wave_words, uint32_t* gscr) {
  NtBatch b = *B;
  NtOut o = *O;
  void* args[] = {&prog, &thr, &b, &o, &tmask, &queue, &len_lo, &len_hi, &claim, &nstatic, &wave_words, &gscr};
  return hipModuleLaunchKernel((hipFunction_t)fn, (unsigned)grid, 1, 1, 256, 1, 1,
                               (unsigned)lds_bytes, stream, args, nullptr);
}

int nt_jit_blocks_per_cu(void* fn, size_t lds_bytes) {
  int nb = 0;
  if (hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&nb, (hipFunction_t)fn, jit_threads(fn), lds_bytes) !=
      hipSuccess)
    return 0;
  return nb;
}

// The calling kernel specialised for the program's patterns (nt_call.h,
// CtCall), or null (and a message) when specialisation is off or failed --
// the caller then launches the ahead-of-time kernel (same results).
void* nt_cjit_get(int device, const NtProgram& P, std::string& err) {
  const char* env = std::getenv("NT_JIT");
  if (env && env[0] == '0') {
    err = "NT_JIT=0";
    return nullptr;
  }
  const std::string src = call_source(P);
  const char* xo = jit_opts();
  const std::string key = std::to_string(device) + "\n" + (xo ? xo : "") + "\n" + src;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_ccache.find(key);
    if (it != g_ccache.end()) {
      if (!it->second.nfn) err = it->second.err;
      return it->second.nfn ? (void*)&it->second : nullptr;
    }
  }
  // built without the lock (seconds): other contexts' lookups go on meanwhile;
  // a build that loses a race to the same key is dropped
  {
    CallEntry e;
    e.split = nt_call_split(P);
    const int nk = e.split ? P.n_pass : 1;
    auto build = [&](const std::string& s) {
      e.nfn = 0;
      if (!compile_module(device, s, e.mod, e.err)) return;
      for (int k = 0; k < nk; ++k) {
        const std::string name = e.split ? "nt_call_jit_p" + std::to_string(k) : std::string("nt_call_jit");
        if (hipModuleGetFunction(&e.fn[k], e.mod, name.c_str()) != hipSuccess) {
          e.err = "hipModuleGetFunction(" + name + ")";
          return;
        }
      }
      e.nfn = nk;
    };
    build(src);
    // Several patterns and TVRs raise the register demand of the unrolled
    // neighbourhood code: at 3 waves/SIMD (168 VGPRs) the c4 set spilled 107
    // VGPRs to scratch and called in 3.6 ms per 2M x 50 kb; at 2 (253 VGPRs, no
    // spill) 2.0 ms.  A kernel that spills more than kCallScratchMax bytes a
    // lane is rebuilt at 2 waves/SIMD (a few spilled registers cost less than
    // the occupancy: the 1-pattern kernels run at 3-4); in the split, only the
    // passes that spill.
    constexpr int kCallScratchMax = 64;
    const bool forced = xo && std::strstr(xo, "NT_CALL_WAVES_P");  // a tuning run sets it
    std::string redo;
    for (int k = 0; k < e.nfn && !forced; ++k) {
      int scratch = 0;
      if (hipFuncGetAttribute(&scratch, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, e.fn[k]) == hipSuccess &&
          scratch > kCallScratchMax)
        redo += e.split ? "#define NT_CALL_WAVES_P" + std::to_string(k) + " 2\n" : "#define NT_CALL_WAVES_PER_EU 2\n";
    }
    if (!redo.empty()) {
      const CallEntry e1 = e;
      build(redo + src);
      if (e.nfn) {
        (void)hipModuleUnload(e1.mod);
      } else {
        e = e1;
      }
    }
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_ccache.find(key);
    if (it == g_ccache.end()) {
      it = g_ccache.emplace(key, e).first;
    } else if (e.mod) {
      (void)hipModuleUnload(e.mod);
    }
    if (!it->second.nfn) err = it->second.err;
    return it->second.nfn ? (void*)&it->second : nullptr;
  }
}

// The specialised calling of batch B (h from nt_cjit_get): the one kernel
// with np <= 2 ? 2 : 4 lanes a read, or a kernel per pass with a lane a read
// and the flag combine after them.  cu_count bounds the grid (64 blocks a CU).
hipError_t nt_cjit_launch(void* h, int np, int cu_count, hipStream_t stream, const NtProgram* prog,
                          const NtBatch* B, const NtOut* O, const uint64_t* tmask, const uint32_t* thr,
                          uint32_t thr_size, int fix_last) {
  const CallEntry& e = *static_cast<const CallEntry*>(h);
  NtBatch b = *B;
  NtOut o = *O;
  void* args[] = {&prog, &b, &o, &tmask, &thr, &thr_size, &fix_last};
  const uint64_t reads = B->list ? B->n_list : B->n_reads;
  const uint64_t lanes = e.split ? reads : reads * (np <= 2 ? 2u : 4u);
  uint64_t grid = (lanes + 255) / 256;
  if (grid > (uint64_t)cu_count * 64) grid = (uint64_t)cu_count * 64;
  if (grid < 1) grid = 1;
  for (int k = 0; k < e.nfn; ++k) {
    const hipError_t r = hipModuleLaunchKernel(e.fn[k], (unsigned)grid, 1, 1, 256, 1, 1, 0, stream, args, nullptr);
    if (r != hipSuccess) return r;
  }
  return e.split ? nt_dev_launch_combine(B, O, np, (int)grid, stream) : hipSuccess;
}

// Fill the on-disk cache with the program's code objects (the scan module and
// the calling kernel, at the default occupancy and at the 2-waves/SIMD
// fallback for spilling builds) without a device: __graft_entry__.build()
// does this for the benchmark's pattern sets, so a fresh GPU box skips hiprtc.
int nt_jit_prebuild_program(const NtProgram& P, const std::string& arch) {
  const std::string a = "--offload-arch=" + arch;
  std::vector<char> code;
  std::string err;
  if (!get_code(a, jit_source(P), code, err)) return -7;
  const std::string cs = call_source(P);
  if (!get_code(a, cs, code, err)) return -7;
  // the spill fallbacks a GPU may ask for (nt_cjit_get): every kernel, or the
  // split's TVR pass alone, at 2 waves/SIMD
  if (nt_call_split(P)) {
    if (P.n_pass == 3 && !get_code(a, "#define NT_CALL_WAVES_P2 2\n" + cs, code, err)) return -7;
    std::string all;
    for (int k = 0; k < P.n_pass; ++k) all += "#define NT_CALL_WAVES_P" + std::to_string(k) + " 2\n";
    if (!get_code(a, all + cs, code, err)) return -7;
  } else if (!get_code(a, "#define NT_CALL_WAVES_PER_EU 2\n" + cs, code, err)) {
    return -7;
  }
  return 0;
}
