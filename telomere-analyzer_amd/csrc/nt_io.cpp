// nt_io.cpp -- streaming FASTA/FASTQ(.gz) reader in nrec-record chunks
// (SURVEY §8(f) row 1): the host ingest of run_future_worker_chuncks
// (NanoTel.R:2171-2216), i.e. XVector's open_input_files + readDNAStringSet(
// files, nrec = nrec, format = format).
//
//  * input_path is a file, or a directory whose files are listed recursively
//    and sorted by full path (dir(full.names = TRUE, recursive = TRUE),
//    NanoTel.R:2176-2178); dot-files and dot-directories are left out, as
//    dir()'s all.files = FALSE does; the files form ONE record stream, a chunk
//    may span files;
//  * gzip is transparent (zlib gzread also reads plain files);
//  * FASTA: '>' starts a record whose name is the rest of the header line;
//    sequence lines are concatenated (line breaks and '\r' dropped, blank
//    lines skipped); FASTQ: 4-line records '@name', sequence, '+...', quality
//    (quality dropped);
//  * letters are kept as they are: validation against DNA_ALPHABET happens in
//    nt_pack_count (NT_E_LETTER), as readDNAStringSet would fail;
//  * a multi-file input (a run directory of fastq.gz parts) is inflated by a
//    few worker threads, files ahead of the parser, each into memory (zlib
//    inflates one stream on one core; the parts are independent), and parsed
//    in order from there.  A single file is streamed.
#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>
#include <sys/stat.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "nanotel.h"

// zlib reports a truncated stream as end of file plus an error state
static bool gz_failed(gzFile g) {
  int e = Z_OK;
  gzerror(g, &e);
  return e != Z_OK && e != Z_STREAM_END;
}

// Inflated files and stream windows live in anonymous mappings that are
// reused, not unmapped: freeing a gigabyte of pages (munmap) costs ~0.1 s of
// kernel time and holds the process's mm lock, which the HIP runtime's own
// calls wait on -- a 16-part fastq.gz run (16 GB inflated) spent 0.7 s of
// reader time unmapping and its context teardown waited 0.3-0.7 s behind it
// (2.6 s read wait and 0.3-0.6 s teardown with the unmaps, 1.9 s and 2 ms
// without).  The process keeps up to NT_READER_POOL_GB (default 32 / local ranks) of them for
// the next parts and the next reader; a buffer grows with mremap (the page
// tables move, nothing is copied).
struct MPool {
  std::mutex mu;
  std::vector<std::pair<char*, size_t>> free;
  size_t bytes = 0, limit = 0;
  MPool() {
    // default 32 GB a node: one process per GPU splits it over the local ranks
    double gb = 32.0;
    if (const char* w = std::getenv("LOCAL_WORLD_SIZE"))
      if (std::atoi(w) > 1) gb /= std::atoi(w);
    const char* v = std::getenv("NT_READER_POOL_GB");
    limit = (size_t)((v ? std::atof(v) : gb) * (double)(1ull << 30));
  }
  char* take(size_t want, size_t& cap) {
    std::lock_guard<std::mutex> lk(mu);
    size_t best = free.size();
    for (size_t i = 0; i < free.size(); ++i)
      if (free[i].second >= want && (best == free.size() || free[i].second < free[best].second)) best = i;
    if (best == free.size() && !free.empty()) {  // none big enough: the biggest, grown by the caller
      best = 0;
      for (size_t i = 1; i < free.size(); ++i)
        if (free[i].second > free[best].second) best = i;
    }
    if (best == free.size()) return nullptr;
    char* p = free[best].first;
    cap = free[best].second;
    bytes -= cap;
    free.erase(free.begin() + (ptrdiff_t)best);
    return p;
  }
  void give(char* p, size_t cap) {
    {
      std::lock_guard<std::mutex> lk(mu);
      if (bytes + cap <= limit) {
        free.emplace_back(p, cap);
        bytes += cap;
        return;
      }
    }
    constexpr size_t kStep = 256u << 20;  // (over the limit: unmapped in steps, the lock released between)
    for (size_t off = 0; off < cap; off += kStep) munmap(p + off, std::min(kStep, cap - off));
  }
};
static MPool& mpool() {
  static MPool* p = new MPool;  // (never destroyed: the mappings go with the process)
  return *p;
}

struct MBuf {
  char* p = nullptr;
  size_t n = 0, cap = 0;
  MBuf() = default;
  MBuf(const MBuf&) = delete;
  MBuf& operator=(const MBuf&) = delete;
  MBuf(MBuf&& o) noexcept { swap(o); }
  MBuf& operator=(MBuf&& o) noexcept {
    if (this != &o) {
      release();
      swap(o);
    }
    return *this;
  }
  ~MBuf() { release(); }
  char* data() { return p; }
  const char* data() const { return p; }
  size_t size() const { return n; }
  bool reserve(size_t want) {
    if (want <= cap) return true;
    const size_t c = (want + (2u << 20) - 1) & ~((size_t)(2u << 20) - 1);  // 2 MB steps
    if (!p) p = mpool().take(c, cap);
    if (c <= cap) return true;
    void* q = p ? mremap(p, cap, c, MREMAP_MAYMOVE) : mmap(nullptr, c, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (q == MAP_FAILED) return false;
    p = (char*)q;
    cap = c;
    return true;
  }
  bool resize(size_t m) {
    if (!reserve(m)) return false;
    n = m;
    return true;
  }
  void swap(MBuf& o) {
    std::swap(p, o.p);
    std::swap(n, o.n);
    std::swap(cap, o.cap);
  }
  void release() {
    if (p) mpool().give(p, cap);
    p = nullptr;
    n = cap = 0;
  }
};

// gzip's ISIZE (the uncompressed size mod 2^32 of the last member): a
// capacity hint for a part inflated whole
static size_t gz_isize_hint(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return 0;
  unsigned char b[4] = {0, 0, 0, 0};
  size_t hint = 0;
  if (std::fseek(f, -4, SEEK_END) == 0 && std::fread(b, 1, 4, f) == 4)
    hint = (size_t)b[0] | ((size_t)b[1] << 8) | ((size_t)b[2] << 16) | ((size_t)b[3] << 24);
  std::fclose(f);
  return hint;
}

// Whole-file inflation of the next files of a multi-file input, ahead of the
// parser: worker threads take files in order, at most `window` beyond the one
// being parsed; the parser waits for its file's buffer.
struct Prefetcher {
  struct Slot {
    bool done = false, plain = false;  // plain: not gzip, the parser reads it itself (parallel pread)
    std::string err;
    MBuf data;
  };
  std::vector<std::string> files_;  // the files in the order the parser takes them (the reader's plan)
  const std::vector<std::string>* files = nullptr;
  std::vector<Slot> slots;
  size_t next = 0, consumed = 0, window = 1, freed = 0;
  bool stop = false;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::thread> workers;

  void start(std::vector<std::string> f, unsigned n_threads) {
    files_ = std::move(f);
    files = &files_;
    slots.resize(files_.size());
    window = n_threads;
    for (unsigned t = 0; t < n_threads; ++t) workers.emplace_back([this] { run(); });
  }
  void run() {
    for (;;) {
      size_t i;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || (next < files->size() && next < consumed + window); });
        if (stop) return;
        i = next++;
      }
      Slot sl;
      unsigned char mg[2] = {0, 0};
      if (FILE* f = std::fopen((*files)[i].c_str(), "rb")) {
        sl.plain = std::fread(mg, 1, 2, f) != 2 || mg[0] != 0x1f || mg[1] != 0x8b;
        std::fclose(f);
      }
      gzFile g = sl.plain ? nullptr : gzopen((*files)[i].c_str(), "rb");
      if (sl.plain) {
      } else if (!g) {
        sl.err = "cannot open " + (*files)[i];
      } else {
        gzbuffer(g, 1 << 20);
        size_t used = 0;
        (void)sl.data.resize(gz_isize_hint((*files)[i]) + (4u << 20));  // (a hint: grows if it is short)
        for (;;) {
          if (sl.data.size() - used < (4u << 20) && !sl.data.resize(std::max<size_t>(8u << 20, sl.data.size() * 2))) {
            sl.err = "out of memory inflating " + (*files)[i];
            break;
          }
          const int n = gzread(g, sl.data.data() + used, (unsigned)std::min<size_t>(sl.data.size() - used, 1u << 30));
          if (n < 0 || (n == 0 && gz_failed(g))) {
            sl.err = "read error in " + (*files)[i];
            break;
          }
          if (n == 0) break;
          used += (size_t)n;
        }
        sl.data.resize(used);
        gzclose(g);
      }
      sl.done = true;
      {
        std::lock_guard<std::mutex> lk(mu);
        slots[i] = std::move(sl);
      }
      cv.notify_all();
    }
  }
  // the inflated file i (waits for it); releases the window for one more file
  bool take(size_t i, MBuf& out, bool& plain, std::string& err) {
    std::unique_lock<std::mutex> lk(mu);
    consumed = i + 1;
    for (; freed < i; ++freed) slots[freed].data.release();  // passed over by a seek
    cv.notify_all();
    cv.wait(lk, [&] { return slots[i].done; });
    if (!slots[i].err.empty()) {
      err = slots[i].err;
      return false;
    }
    plain = slots[i].plain;
    if (plain) return true;
    out.swap(slots[i].data);
    slots[i].data.release();
    return true;
  }
  ~Prefetcher() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : workers) t.join();
  }
};

// A buffer records point into: an inflated file or stream window (owned
// bytes) or a read-only mapping of a plain file.  Shared: the chunk stores
// that hold pointers into a buffer keep it alive (a chunk stays valid through
// the next nt_reader_next call).
struct RBuf {
  MBuf own;
  void* map = nullptr;
  size_t map_len = 0;
  const char* data = nullptr;
  size_t size = 0;
  ~RBuf() {
    if (map) munmap(map, map_len);
  }
};

struct nt_reader {
  std::vector<std::string> files;
  // the files in the order they are read: all of them, or the plan of a rank
  // of a sharded run (nt_reader_plan: only the files its chunks touch)
  std::vector<uint64_t> order;
  size_t file_idx = 0;  // next position in `order` to open
  uint64_t cur_file = ~0ull;  // the open file (index into files)
  uint64_t rec_in_file = 0;   // records parsed in it so far
  int format = 0;       // 0 fasta, 1 fastq
  unsigned pf_threads = 0;  // gzip parts inflated ahead (multi-file input), started at the first open
  bool started = false;
  // sharded ingest: plain files' sizes and offsets in the concatenated stream,
  // the record starts of this rank's byte range (nt_reader_shard_range)
  std::vector<uint64_t> fsize, fbase;
  std::vector<uint64_t> shard_pos;
  // bytes the parser walked over (records, kept or skipped) and bytes inflated
  uint64_t bytes_parsed = 0, bytes_inflated = 0;
  size_t rec_at = 0;  // header offset (in the window) of the last record parsed
  // FASTQ fast path (a mapped plain file): records indexed in parallel slices
  // without reading the quality lines (fq_index_slice); fq_mode 1 = on for
  // the open file, 0 = off (the line parser)
  struct FqRec {
    uint64_t hdr, name_at, name_len, seq_at, seq_len, end;
  };
  std::vector<FqRec> fq;
  size_t fq_i = 0;
  uint64_t fq_scan = 0;
  int fq_mode = 0;
  // the next slice's byte cap: 1 GB when reading on, kSliceSeek after a seek
  // that left the index (a rank's block may be far smaller than a slice:
  // indexing 1 GB of other ranks' records per seek undid the sharding), then
  // doubling
  uint64_t fq_slice = 0;
  // the current file's bytes: a mapping of the whole plain file, a whole gzip
  // part inflated ahead (Prefetcher), or windows of a gzip stream (serial inflate)
  gzFile gz = nullptr;
  bool active = false;   // a file is open
  bool src_eof = true;   // no bytes of the current file beyond win[end)
  std::unique_ptr<Prefetcher> pf;
  // the window: bytes [pos, end) of win not yet parsed; nl = offsets of the
  // '\n' in [pos, scan) (indexed lazily, in slices), nl[nl_i] the first one at
  // or after pos
  std::shared_ptr<RBuf> win;
  size_t pos = 0, end = 0, scan = 0;
  std::vector<uint64_t> nl;
  size_t nl_i = 0;
  std::string err;
  // chunk storage, two slots used in turn: a chunk stays valid through the
  // next nt_reader_next call (so the caller can read chunk k+1 on another
  // thread while it still scans chunk k).  Names and single-line sequences
  // point into the buffers (refs); multi-line FASTA sequences are joined in
  // seqs_blob (seq_off = blob offset, marked by seq_blob).
  struct Store {
    std::string seqs_blob;
    std::vector<uint64_t> seq_off;
    std::vector<uint8_t> seq_blob;
    std::vector<const char*> name_ptr, seq_ptr;
    std::vector<uint64_t> name_len, seq_len;
    std::vector<std::shared_ptr<RBuf>> refs;
  };
  std::vector<Store> store = std::vector<Store>(2);  // a ring: the last store.size() chunks stay valid
  size_t cur = 0;
  Store& c() { return store[cur]; }
  // nt_reader_skip's lengths (two in turn: valid through the next skip call;
  // skips do not take a chunk store)
  std::vector<uint64_t> skip_len[2];
  int skip_cur = 0;
  // the current record's multi-line FASTA pieces (offset, length in win)
  std::vector<std::pair<uint64_t, uint64_t>> pieces;
  uint64_t records_total = 0;
};

namespace {

constexpr size_t kWindow = 64u << 20;  // gzip stream window / index slice (grows for a larger record)

unsigned host_threads() {
  unsigned nt = std::thread::hardware_concurrency();
  nt = nt == 0 ? 1u : nt;
  // one process per GPU: the ranks of a node share its cores; at most 16 a
  // rank (a GPU's share of the host on the MI355X nodes)
  if (const char* w = std::getenv("LOCAL_WORLD_SIZE")) {
    const int k = atoi(w);
    if (k > 1) nt = std::max(1u, nt / (unsigned)k);
  }
  nt = std::min(nt, 16u);
  if (const char* v = std::getenv("NT_READER_PARSE_THREADS")) nt = (unsigned)std::max(1, atoi(v));
  return nt;
}

template <class F>
void par(unsigned n, F&& f) {
  if (n <= 1) {
    if (n) f(0u);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned t = 1; t < n; ++t) th.emplace_back([&f, t] { f(t); });
  f(0u);
  for (auto& x : th) x.join();
}

void list_files(const std::string& path, std::vector<std::string>& out) {
  DIR* d = opendir(path.c_str());
  if (!d) return;
  while (dirent* e = readdir(d)) {
    const std::string n = e->d_name;
    // dir(all.files = FALSE): names starting with '.' (".", "..", ".DS_Store",
    // AppleDouble "._x.fastq.gz", hidden directories) are not listed
    if (n.empty() || n[0] == '.') continue;
    const std::string full = path + "/" + n;
    struct stat st;
    if (stat(full.c_str(), &st) != 0) continue;
    if (S_ISDIR(st.st_mode)) list_files(full, out);
    else out.push_back(full);
  }
  closedir(d);
}

bool is_gzip(const std::string& path) {
  unsigned char m[2] = {0, 0};
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  const size_t k = std::fread(m, 1, 2, f);
  std::fclose(f);
  return k == 2 && m[0] == 0x1f && m[1] == 0x8b;
}

void close_source(nt_reader* r) {
  if (r->gz) gzclose(r->gz);
  r->gz = nullptr;
  r->active = false;
}

// Index the '\n' of the next slice of the window, [scan, scan + kWindow) or
// to its end: parallel memchr (which also faults a mapping's pages in on all
// host threads).  Returns false when the window is indexed to its end.
bool index_more(nt_reader* r) {
  const size_t a = r->scan, b = std::min(r->end, r->scan + kWindow);
  if (b <= a) return false;
  if (r->nl_i > 0) {  // drop the consumed entries
    r->nl.erase(r->nl.begin(), r->nl.begin() + (ptrdiff_t)r->nl_i);
    r->nl_i = 0;
  }
  const char* base = r->win->data;
  auto scan_range = [base](size_t x, size_t y, std::vector<uint64_t>& out) {
    const char* p = base + x;
    const char* e = base + y;
    while (p < e) {
      const char* q = (const char*)memchr(p, '\n', (size_t)(e - p));
      if (!q) break;
      out.push_back((uint64_t)(q - base));
      p = q + 1;
    }
  };
  const unsigned nt = (b - a) >= (4u << 20) ? host_threads() : 1u;
  if (nt == 1) {
    scan_range(a, b, r->nl);
  } else {
    std::vector<std::vector<uint64_t>> part(nt);
    par(nt, [&](unsigned t) { scan_range(a + (b - a) * t / nt, a + (b - a) * (t + 1) / nt, part[t]); });
    for (auto& v : part) r->nl.insert(r->nl.end(), v.begin(), v.end());
  }
  r->scan = b;
  return true;
}

// More of the current file: index the window further, or (gzip stream)
// inflate the next window -- a new buffer that starts with the unparsed
// bytes [pos, end) (records of the current chunk may point into the old
// one).  Returns false when nothing more can come (end of file, or error).
bool more(nt_reader* r) {
  if (r->scan < r->end) return index_more(r);
  if (r->src_eof || !r->active) return false;
  const size_t keep = r->end - r->pos;
  size_t cap = std::max(kWindow, 2 * keep);
  auto nb = std::make_shared<RBuf>();
  if (!nb->own.resize(cap)) {
    r->err = "out of memory reading " + r->files[r->cur_file];
    r->src_eof = true;
    return false;
  }
  if (keep) std::memcpy(nb->own.data(), r->win->data + r->pos, keep);
  size_t got = keep;
  while (got < cap) {
    const int n = gzread(r->gz, nb->own.data() + got, (unsigned)std::min<size_t>(cap - got, 1u << 30));
    if (n < 0 || (n == 0 && gz_failed(r->gz))) {  // corrupt or truncated gzip stream
      r->err = "read error in " + r->files[r->cur_file];
      r->src_eof = true;
      return false;
    }
    if (n == 0) {
      r->src_eof = true;
      break;
    }
    got += (size_t)n;
  }
  r->bytes_inflated += got - keep;
  nb->data = nb->own.data();
  nb->size = got;
  for (size_t i = r->nl_i; i < r->nl.size(); ++i) r->nl[i] -= r->pos;
  r->scan -= r->pos;
  r->win = nb;
  r->end = got;
  r->pos = 0;
  return got > keep;
}

// The reader's first open: the inflate-ahead workers of a multi-file input
// start on the files of the plan (all files unless nt_reader_plan named some).
void start(nt_reader* r) {
  if (r->started) return;
  r->started = true;
  if (r->pf_threads > 0 && r->order.size() > 1) {
    std::vector<std::string> paths;
    for (uint64_t f : r->order) paths.push_back(r->files[f]);
    r->pf.reset(new Prefetcher());
    r->pf->start(std::move(paths), r->pf_threads);
  }
}

// the FASTQ fast path's state for a new position of the open file
constexpr uint64_t kSliceMax = 1ull << 30, kSliceSeek = 16ull << 20;

void fq_reset(nt_reader* r, uint64_t pos, bool mapped, uint64_t slice = kSliceMax) {
  r->fq.clear();
  r->fq_i = 0;
  r->fq_scan = pos;
  r->fq_slice = slice;
  const char* v = std::getenv("NT_READER_FQ_FAST");  // 0: the line parser for FASTQ too
  const bool off = v && v[0] == '0';
  r->fq_mode = (r->format == 1 && mapped && !off) ? 1 : 0;
}

bool open_next(nt_reader* r) {
  close_source(r);
  r->fq_mode = 0;
  r->win.reset();
  r->pos = r->end = r->scan = 0;
  r->nl.clear();
  r->nl_i = 0;
  r->cur_file = ~0ull;
  r->rec_in_file = 0;
  start(r);
  if (!r->err.empty() || r->file_idx >= r->order.size()) return false;
  r->cur_file = r->order[r->file_idx++];
  const std::string& path = r->files[r->cur_file];
  auto b = std::make_shared<RBuf>();
  if (r->pf) {  // a gzip part inflated ahead by the workers: parse straight from memory
    bool plain = false;
    if (!r->pf->take(r->file_idx - 1, b->own, plain, r->err)) return false;
    if (!plain) {
      r->bytes_inflated += b->own.size();
      b->data = b->own.data();
      b->size = b->own.size();
      r->win = b;
      r->end = b->size;
      r->src_eof = true;
      r->active = true;
      return true;
    }
  }
  if (!is_gzip(path)) {  // a plain file: mapped whole (no copy; pages fault in during the index)
    const int fd = ::open(path.c_str(), O_RDONLY);
    struct stat st;
    if (fd < 0 || fstat(fd, &st) != 0) {
      if (fd >= 0) ::close(fd);
      r->err = "cannot open " + path;
      return false;
    }
    if (st.st_size > 0) {
      void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (m == MAP_FAILED) {
        ::close(fd);
        r->err = "cannot map " + path;
        return false;
      }
      (void)madvise(m, (size_t)st.st_size, MADV_SEQUENTIAL);
      b->map = m;
      b->map_len = (size_t)st.st_size;
      b->data = (const char*)m;
      b->size = (size_t)st.st_size;
    }
    ::close(fd);
    r->win = b;
    r->end = b->size;
    r->src_eof = true;
    r->active = true;
    fq_reset(r, 0, b->map != nullptr);
    return true;
  }
  r->gz = gzopen(path.c_str(), "rb");
  if (!r->gz) {
    r->err = "cannot open " + path;
    return false;
  }
  gzbuffer(r->gz, 1 << 20);
  r->win = b;  // empty: the first more() inflates
  r->src_eof = false;
  r->active = true;
  return true;
}

// Line cursor over the window: (p, i) = byte offset and index into nl of the
// next '\n' at or after p.
struct Cur {
  size_t p, i;
};

// The next line at the cursor: [ls, le) without '\n' / '\r'.  false when the
// window holds no complete line there: more bytes (or index) may come (need =
// true), or the file is exhausted (need = false).  At the end of a file the
// last, unterminated line counts.
bool next_line(const nt_reader* r, Cur& c, size_t& ls, size_t& le, bool& need) {
  need = false;
  if (c.p >= r->end) {
    need = !r->src_eof;
    return false;
  }
  ls = c.p;
  if (c.i < r->nl.size()) {
    le = (size_t)r->nl[c.i];
    c.p = le + 1;
    ++c.i;
  } else {
    if (r->scan < r->end || !r->src_eof) {
      need = true;
      return false;
    }
    le = r->end;
    c.p = r->end;
  }
  if (le > ls && r->win->data[le - 1] == '\r') --le;
  return true;
}

// A record was parsed: the cursor moves past it (rec_at = its header line's
// offset in the window; the bytes walked over count as parsed).
void commit(nt_reader* r, const Cur& c, size_t hdr) {
  r->bytes_parsed += c.p - r->pos;
  r->pos = c.p;
  r->nl_i = c.i;
  r->rec_at = hdr;
  ++r->rec_in_file;
}

// One record from the window at the committed cursor, appended to the chunk
// store (or, when lens_only, its sequence length only).  Returns 1 = a
// record, 0 = end of this file, -1 = error, 2 = incomplete (more() and retry).
int parse_record(nt_reader* r, bool lens_only, std::vector<uint64_t>* skip_lens) {
  Cur c{r->pos, r->nl_i};
  size_t ls = 0, le = 0;
  bool need = false;
  const char* b = r->win->data;
  auto& S = r->c();
  if (r->format == 0) {
    for (;;) {  // the header (lines before the first one are skipped)
      if (!next_line(r, c, ls, le, need)) return need ? 2 : 0;
      if (le > ls && b[ls] == '>') break;
    }
    const size_t hdr = ls, name_at = ls + 1, name_len = le - ls - 1;
    r->pieces.clear();
    uint64_t len = 0;
    for (;;) {  // sequence lines up to the next header or the end of the file
      Cur save = c;
      if (!next_line(r, c, ls, le, need)) {
        if (need) return 2;
        break;
      }
      if (le == ls || b[ls] == ';') continue;  // blank and ';' comment lines are dropped
      if (b[ls] == '>') {
        c = save;  // the next record's header
        break;
      }
      len += le - ls;
      r->pieces.emplace_back(ls, le - ls);
    }
    commit(r, c, hdr);
    if (lens_only) {
      skip_lens->push_back(len);
      return 1;
    }
    S.seq_len.push_back(len);
    S.name_ptr.push_back(b + name_at);
    S.name_len.push_back(name_len);
    if (r->pieces.size() <= 1) {  // one line: points into the buffer
      S.seq_ptr.push_back(r->pieces.empty() ? b + name_at : b + r->pieces[0].first);
      S.seq_blob.push_back(0);
      S.seq_off.push_back(0);
    } else {  // wrapped: joined in the store's blob
      S.seq_ptr.push_back(nullptr);
      S.seq_blob.push_back(1);
      S.seq_off.push_back(S.seqs_blob.size());
      for (auto& pc : r->pieces) S.seqs_blob.append(b + pc.first, pc.second);
    }
    return 1;
  }
  // FASTQ: '@' name, the sequence line, '+' line, quality lines up to the sequence's length
  for (;;) {
    if (!next_line(r, c, ls, le, need)) return need ? 2 : 0;
    if (le == ls) continue;
    if (b[ls] != '@') {
      r->err = "malformed FASTQ record (expected '@')";
      return -1;
    }
    break;
  }
  const size_t hdr = ls, name_at = ls + 1, name_len = le - ls - 1;
  auto malformed = [&] {
    r->err = "malformed FASTQ record '" + std::string(b + name_at, name_len) + "'";
    return -1;
  };
  size_t ss = 0, se = 0;
  if (!next_line(r, c, ss, se, need)) return need ? 2 : malformed();
  if (!next_line(r, c, ls, le, need) || le == ls || b[ls] != '+') return need ? 2 : malformed();
  uint64_t ql = 0;
  const uint64_t sl = se - ss;
  while (ql < sl) {  // quality may in principle wrap
    if (!next_line(r, c, ls, le, need)) {
      if (need) return 2;
      break;
    }
    ql += le - ls;
  }
  commit(r, c, hdr);
  if (lens_only) {
    skip_lens->push_back(sl);
    return 1;
  }
  S.seq_len.push_back(sl);
  S.name_ptr.push_back(b + name_at);
  S.name_len.push_back(name_len);
  S.seq_ptr.push_back(b + ss);
  S.seq_blob.push_back(0);
  S.seq_off.push_back(0);
  return 1;
}

size_t resync(const char* d, size_t n, size_t o, int format);
size_t nl_at(const char* d, size_t n, size_t p);

// offset of the first non-blank line at or after p (blank: "\n" or "\r\n")
size_t skip_blank(const char* d, size_t n, size_t p) {
  for (;;) {
    if (p < n && d[p] == '\n') ++p;
    else if (p + 1 < n && d[p] == '\r' && d[p + 1] == '\n') p += 2;
    else return p;
  }
}

// One FASTQ record whose header is at p (p past any blank lines) with the
// line parser's semantics (parse_record): '@' name, the sequence line, a '+'
// line, quality lines up to the sequence's length -- a single quality line
// of exactly that length is skipped without being read (its newline is
// checked), otherwise its lines are walked.  Returns 1 (rec, next = the
// offset after the record's last line), 0 (p at the end), -1 malformed.
int fq_parse_one(const char* d, size_t n, size_t p, nt_reader::FqRec& rec, size_t& next) {
  if (p >= n) return 0;
  if (d[p] != '@') return -1;
  const size_t eh = nl_at(d, n, p);
  if (eh >= n) return -1;
  size_t ne = eh;
  if (ne > p + 1 && d[ne - 1] == '\r') --ne;
  const size_t s0 = eh + 1, es = nl_at(d, n, s0);
  size_t se = es;
  if (se > s0 && d[se - 1] == '\r') --se;
  if (es >= n) return -1;  // no '+' line
  const size_t pl = es + 1;
  if (pl >= n || d[pl] != '+') return -1;
  const size_t ep = nl_at(d, n, pl);
  const uint64_t sl = se - s0;
  size_t c = ep >= n ? n : ep + 1;
  if (sl > 0 && c < n) {
    const size_t qe = c + sl;
    // one quality line of exactly sl letters: a line end at qe, no line end
    // inside [c, qe) (a wrapped quality whose lines and newlines add up to
    // sl), no '\r' at qe - 1 (a CRLF line of sl - 1 letters) -- otherwise the
    // line walk below, which is the line parser's (parse_record): both then
    // see the same lines and reject the same malformed records
    const bool one_line = qe <= n && d[qe - 1] != '\r' && !std::memchr(d + c, '\n', sl);
    if (one_line && qe == n) {
      c = n;
    } else if (one_line && qe < n && d[qe] == '\n') {
      c = qe + 1;
    } else if (one_line && qe + 1 < n && d[qe] == '\r' && d[qe + 1] == '\n') {
      c = qe + 2;
    } else {  // wrapped (or longer) quality: its lines, up to the sequence's length
      uint64_t ql = 0;
      while (ql < sl && c < n) {
        const size_t e = nl_at(d, n, c);
        size_t le = e;
        if (le > c && d[le - 1] == '\r') --le;
        ql += le - c;
        c = e >= n ? n : e + 1;
      }
    }
  }
  rec.hdr = p;
  rec.name_at = p + 1;
  rec.name_len = ne - p - 1;
  rec.seq_at = s0;
  rec.seq_len = sl;
  rec.end = c;
  next = c;
  return 1;
}

// Index the records that start in the next slice of the mapped FASTQ file
// (up to 1 GB) on the host threads: each thread resynchronises in its part
// (an '@' line whose second next line starts with '+'), parses records up to
// its part's end, and the parts must chain (thread t's first record is where
// thread t - 1 stopped).  Returns 1 (records appended; fq_scan moved on), 0
// (the file is done), -1 (a part did not chain or a record is malformed: the
// caller goes on with the line parser from fq_scan).
int fq_index_slice(nt_reader* r) {
  const char* d = r->win->data;
  const size_t n = r->end;
  const size_t a = skip_blank(d, n, r->fq_scan);
  if (a >= n) return 0;
  const size_t slice = r->fq_slice ? r->fq_slice : kSliceMax;
  r->fq_slice = std::min<uint64_t>(kSliceMax, 2 * slice);
  const size_t b = std::min(n, a + slice);
  const unsigned nt = (b - a) >= (8u << 20) ? host_threads() : 1u;
  struct Part {
    std::vector<nt_reader::FqRec> recs;
    size_t first = 0, next = 0;
    bool bad = false;
  };
  std::vector<Part> part(nt);
  par(nt, [&](unsigned t) {
    Part& P = part[t];
    const size_t lo = a + (b - a) * t / nt, hi = a + (b - a) * (t + 1) / nt;
    size_t p = t == 0 ? a : skip_blank(d, n, resync(d, n, lo, 1));
    P.first = p;
    while (p < hi && p < n) {
      nt_reader::FqRec rec;
      size_t nx = 0;
      const int k = fq_parse_one(d, n, p, rec, nx);
      if (k == 0) break;
      if (k < 0) {
        P.bad = true;
        break;
      }
      P.recs.push_back(rec);
      p = skip_blank(d, n, nx);
    }
    P.next = p;
  });
  for (unsigned t = 0; t < nt; ++t)
    if (part[t].bad || (t && part[t].first != part[t - 1].next)) return -1;
  for (auto& P : part) r->fq.insert(r->fq.end(), P.recs.begin(), P.recs.end());
  r->fq_scan = part[nt - 1].next;
  return 1;
}

// Up to nrec records into the chunk store (or their lengths only); returns
// the count, or -1 on error.
int64_t read_records(nt_reader* r, uint64_t nrec, bool lens_only, std::vector<uint64_t>* skip_lens) {
  auto& S = r->c();
  uint64_t got = 0;
  bool ref = false;  // the chunk holds a reference to the current window
  while (got < nrec) {
    if (!r->active) {
      if (!open_next(r)) break;
      ref = false;
      continue;
    }
    if (r->fq_mode == 1) {  // FASTQ fast path: records from the slice index
      if (r->fq_i < r->fq.size()) {
        const nt_reader::FqRec& q = r->fq[r->fq_i++];
        const char* b = r->win->data;
        r->bytes_parsed += q.end - r->pos;
        r->pos = q.end;
        r->rec_at = q.hdr;
        ++r->rec_in_file;
        ++got;
        if (lens_only) {
          skip_lens->push_back(q.seq_len);
          continue;
        }
        S.seq_len.push_back(q.seq_len);
        S.name_ptr.push_back(b + q.name_at);
        S.name_len.push_back(q.name_len);
        S.seq_ptr.push_back(b + q.seq_at);
        S.seq_blob.push_back(0);
        S.seq_off.push_back(0);
        if (!ref) {
          S.refs.push_back(r->win);
          ref = true;
        }
        continue;
      }
      r->fq.clear();
      r->fq_i = 0;
      const int k = fq_index_slice(r);
      if (k > 0) continue;
      if (k == 0) {  // the file is done
        r->pos = r->end;
        close_source(r);
        continue;
      }
      // the line parser from here on (it reports a malformed record where it is)
      r->fq_mode = 0;
      r->pos = r->scan = (size_t)r->fq_scan;
      r->nl.clear();
      r->nl_i = 0;
      continue;
    }
    const int k = parse_record(r, lens_only, skip_lens);
    if (k == 1) {
      ++got;
      if (!lens_only && !ref) {
        S.refs.push_back(r->win);
        ref = true;
      }
      continue;
    }
    if (k < 0) return -1;
    if (k == 2) {  // incomplete: index further, or inflate the next window
      const RBuf* w = r->win.get();
      if (!more(r) && !r->err.empty()) return -1;
      if (r->win.get() != w) ref = false;
      continue;
    }
    if (!r->err.empty()) return -1;  // k == 0: this file is done
    close_source(r);
  }
  if (!r->err.empty()) return -1;
  return (int64_t)got;
}

}  // namespace

extern "C" {

int nt_reader_open(const char* path, int format, nt_reader** out) {
  if (!path || !out || (format != 0 && format != 1)) return NT_E_ARG;
  *out = nullptr;
  nt_reader* r = new (std::nothrow) nt_reader();
  if (!r) return NT_E_NOMEM;
  struct stat st;
  if (stat(path, &st) != 0) {
    delete r;
    return NT_E_ARG;
  }
  if (S_ISDIR(st.st_mode)) {
    std::string p = path;
    while (p.size() > 1 && p.back() == '/') p.pop_back();
    list_files(p, r->files);
    std::sort(r->files.begin(), r->files.end());
  } else {
    r->files.push_back(path);
  }
  r->format = format;
  r->order.resize(r->files.size());
  for (size_t i = 0; i < r->files.size(); ++i) r->order[i] = i;
  if (r->files.size() > 1) {  // a run directory: inflate gzip parts ahead on worker threads
    unsigned nt = std::thread::hardware_concurrency();
    nt = std::max(1u, std::min(nt == 0 ? 1u : nt, 16u));
    if (const char* v = std::getenv("NT_READER_THREADS")) nt = (unsigned)std::max(0, atoi(v));
    r->pf_threads = nt;
  }
  *out = r;
  return NT_OK;
}

void nt_reader_close(nt_reader* r) {
  if (!r) return;
  close_source(r);
  // unmapping a large input (the page tables of gigabytes) takes milliseconds:
  // done off the caller's path (NT_READER_SYNC_CLOSE: here, e.g. for leak checks)
  if (std::getenv("NT_READER_SYNC_CLOSE")) {
    delete r;
    return;
  }
  std::thread([r] { delete r; }).detach();
}

uint64_t nt_reader_file_count(const nt_reader* r) { return r ? r->files.size() : 0; }

const char* nt_reader_file(const nt_reader* r, uint64_t i) {
  return (r && i < r->files.size()) ? r->files[i].c_str() : nullptr;
}

const char* nt_reader_error(const nt_reader* r) { return r ? r->err.c_str() : "null reader"; }

static void clear_store(nt_reader* r) {
  r->cur = (r->cur + 1) % r->store.size();
  auto& S = r->c();
  S.seqs_blob.clear();
  S.seq_off.clear();
  S.seq_blob.clear();
  S.name_ptr.clear();
  S.seq_ptr.clear();
  S.name_len.clear();
  S.seq_len.clear();
  S.refs.clear();  // the buffers of the chunk store.size() calls back (no longer valid)
}

int nt_reader_keep(nt_reader* r, uint32_t chunks) {
  if (!r || chunks < 2 || chunks > 4096) return NT_E_ARG;
  if (chunks > r->store.size()) {  // the new stores come after the current one in the ring
    r->store.insert(r->store.begin() + (ptrdiff_t)r->cur + 1, chunks - r->store.size(), nt_reader::Store());
  }
  return NT_OK;
}

int64_t nt_reader_next(nt_reader* r, uint64_t nrec, const char* const** names,
                       const uint64_t** name_lens, const char* const** seqs,
                       const uint64_t** seq_lens) {
  if (!r || !names || !name_lens || !seqs || !seq_lens || nrec == 0) return NT_E_ARG;
  clear_store(r);
  const int64_t n = read_records(r, nrec, false, nullptr);
  if (n < 0) return NT_E_ARG;
  auto& S = r->c();
  for (int64_t i = 0; i < n; ++i)  // joined sequences: the blob no longer grows
    if (S.seq_blob[i]) S.seq_ptr[i] = S.seqs_blob.data() + S.seq_off[i];
  *names = S.name_ptr.data();
  *name_lens = S.name_len.data();
  *seqs = S.seq_ptr.data();
  *seq_lens = S.seq_len.data();
  r->records_total += (uint64_t)n;
  return n;
}

int64_t nt_reader_skip(nt_reader* r, uint64_t nrec, const uint64_t** seq_lens) {
  if (!r || !seq_lens || nrec == 0) return NT_E_ARG;
  r->skip_cur ^= 1;
  auto& L = r->skip_len[r->skip_cur];
  L.clear();
  const int64_t n = read_records(r, nrec, true, &L);
  if (n < 0) return NT_E_ARG;
  *seq_lens = L.data();
  r->records_total += (uint64_t)n;
  return n;
}

}  // extern "C"

// ------------------------------------------------------------ sharded ingest
//
// One process per GPU reads its share of the input instead of the whole
// stream: every rank finds where the nrec-record chunks start
// from 1/N of the bytes, then reads only the chunks it scans.
//  * plain files (all of them): rank r indexes bytes [S r / N, S (r+1) / N) of
//    the concatenated files -- it resynchronises at the first record start in
//    its range (FASTA: a '>' line; FASTQ: an '@' line whose second next line
//    starts with '+') and counts the records starting there; the ranks' counts
//    give every record its global index, so the chunk starts are known;
//  * gzip parts (a run directory): a gzip stream can only be inflated from its
//    start, so rank r counts the records of whole files f = r (mod N);
//  * then each rank seeks to its chunks' starts (nt_reader_seek) and reads
//    them with nt_reader_next, visiting only the files its plan names
//    (nt_reader_plan: the inflate-ahead workers take only those).
// A resynchronisation that is not a true record start (a FASTQ quality line
// shaped like a header) shows as a mismatch between rank r's first record and
// the record at which rank r - 1's parse crossed into rank r's range: the
// caller checks first(r) == next(r - 1) and otherwise reads unsharded.
namespace {

size_t nl_at(const char* d, size_t n, size_t p) {  // offset of the '\n' ending the line at p (or n)
  const void* q = p < n ? memchr(d + p, '\n', n - p) : nullptr;
  return q ? (size_t)((const char*)q - d) : n;
}

// first record-start candidate at or after byte o (> 0) of a plain file
size_t resync(const char* d, size_t n, size_t o, int format) {
  size_t p = o;
  if (p > 0 && p < n && d[p - 1] != '\n') {
    const size_t e = nl_at(d, n, p);
    if (e >= n) return n;
    p = e + 1;
  }
  while (p < n) {
    const size_t e1 = nl_at(d, n, p);
    if (format == 0) {
      if (d[p] == '>') return p;
    } else if (d[p] == '@' && e1 + 1 < n) {
      const size_t e2 = nl_at(d, n, e1 + 1);
      if (e2 + 1 < n && d[e2 + 1] == '+') return p;
    }
    if (e1 >= n) return n;
    p = e1 + 1;
  }
  return n;
}

// a temporary reader over some of r's files (no inflate-ahead workers)
void init_like(nt_reader& t, const nt_reader* r) {
  t.files = r->files;
  t.format = r->format;
  t.pf_threads = 0;
  t.order.clear();
}

// first file holding byte x of the concatenated plain files (n if none)
size_t file_at(const nt_reader* r, uint64_t x) {
  for (size_t f = 0; f < r->fsize.size(); ++f)
    if (r->fbase[f] + r->fsize[f] > x) return f;
  return r->fsize.size();
}

}  // namespace

extern "C" {

int nt_reader_layout(nt_reader* r, int* all_plain, uint64_t* total_bytes) {
  if (!r || !all_plain || !total_bytes) return NT_E_ARG;
  r->fsize.assign(r->files.size(), 0);
  r->fbase.assign(r->files.size(), 0);
  int plain = 1;
  uint64_t tot = 0;
  for (size_t f = 0; f < r->files.size(); ++f) {
    struct stat st;
    if (stat(r->files[f].c_str(), &st) != 0) {
      r->err = "cannot open " + r->files[f];
      return NT_E_ARG;
    }
    if (is_gzip(r->files[f])) plain = 0;
    r->fsize[f] = (uint64_t)st.st_size;
    r->fbase[f] = tot;
    tot += (uint64_t)st.st_size;
  }
  *all_plain = plain;
  *total_bytes = tot;
  return NT_OK;
}

int64_t nt_reader_shard_range(nt_reader* r, uint64_t a, uint64_t b, uint64_t* first, uint64_t* next) {
  if (!r || !first || !next || b < a || r->fbase.size() != r->files.size()) return NT_E_ARG;
  const uint64_t S = r->fbase.empty() ? 0 : r->fbase.back() + r->fsize.back();
  r->shard_pos.clear();
  *first = *next = S;
  const size_t f = file_at(r, a);
  if (a >= S || f >= r->files.size()) return 0;
  nt_reader t;
  init_like(t, r);
  for (size_t g = f; g < r->files.size(); ++g) t.order.push_back(g);
  if (!open_next(&t)) {
    r->err = t.err;
    return NT_E_ARG;
  }
  // a range that starts inside a file resynchronises; one that starts at a
  // file's first byte parses it as the unsharded reader does (errors included)
  const uint64_t o = a - r->fbase[f];
  const size_t p = o == 0 ? 0 : resync(t.win->data, t.end, (size_t)o, t.format);
  t.pos = t.scan = p;
  std::vector<uint64_t> lens;
  bool have_first = false;
  for (;;) {
    const int k = parse_record(&t, true, &lens);
    if (k == 1) {
      const uint64_t x = r->fbase[t.cur_file] + t.rec_at;
      if (!have_first) {
        *first = x;
        have_first = true;
      }
      if (x >= b) {
        *next = x;
        break;
      }
      r->shard_pos.push_back(x);
      if (lens.size() > 4096) lens.clear();
      continue;
    }
    if (k < 0) {
      r->err = t.err;
      return NT_E_ARG;
    }
    if (k == 2) {
      if (!more(&t) && !t.err.empty()) {
        r->err = t.err;
        return NT_E_ARG;
      }
      continue;
    }
    if (!t.err.empty()) {
      r->err = t.err;
      return NT_E_ARG;
    }
    if (!open_next(&t)) {  // end of the stream
      if (!t.err.empty()) {
        r->err = t.err;
        return NT_E_ARG;
      }
      break;
    }
  }
  r->bytes_parsed += t.bytes_parsed;
  return (int64_t)r->shard_pos.size();
}

int64_t nt_reader_shard_positions(const nt_reader* r, const uint64_t** pos) {
  if (!r || !pos) return NT_E_ARG;
  *pos = r->shard_pos.data();
  return (int64_t)r->shard_pos.size();
}

int nt_reader_count_files(nt_reader* r, const uint64_t* files, uint64_t n, uint64_t* counts) {
  if (!r || (n && (!files || !counts))) return NT_E_ARG;
  for (uint64_t i = 0; i < n; ++i)
    if (files[i] >= r->files.size()) return NT_E_ARG;
  std::atomic<uint64_t> next{0}, parsed{0}, inflated{0};
  std::mutex mu;
  std::string err;
  const unsigned nt = (unsigned)std::min<uint64_t>(host_threads(), n);
  par(nt, [&](unsigned) {
    for (uint64_t i = next++; i < n; i = next++) {
      nt_reader t;
      init_like(t, r);
      t.order.push_back(files[i]);
      std::vector<uint64_t> lens;
      uint64_t c = 0;
      for (;;) {
        lens.clear();
        const int64_t k = read_records(&t, 1u << 16, true, &lens);
        if (k < 0) {
          std::lock_guard<std::mutex> lk(mu);
          if (err.empty()) err = t.err;
          return;
        }
        if (k == 0) break;
        c += (uint64_t)k;
      }
      counts[i] = c;
      parsed += t.bytes_parsed;
      inflated += t.bytes_inflated;
    }
  });
  r->bytes_parsed += parsed;
  r->bytes_inflated += inflated;
  if (!err.empty()) {
    r->err = err;
    return NT_E_ARG;
  }
  return NT_OK;
}

int nt_reader_plan(nt_reader* r, const uint64_t* files, uint64_t n) {
  if (!r || (n && !files)) return NT_E_ARG;
  if (r->started) return NT_E_STATE;
  for (uint64_t i = 0; i < n; ++i)
    if (files[i] >= r->files.size() || (i && files[i] <= files[i - 1])) return NT_E_ARG;
  r->order.assign(files, files + n);
  return NT_OK;
}

int nt_reader_seek(nt_reader* r, int mode, uint64_t a, uint64_t b) {
  if (!r || (mode != 0 && mode != 1)) return NT_E_ARG;
  start(r);
  uint64_t f = 0, off = 0, skip = 0;
  if (mode == 0) {  // byte a of the concatenated plain files
    if (r->fbase.size() != r->files.size()) return NT_E_ARG;
    f = file_at(r, a);
    if (f >= r->files.size()) {  // the end of the stream
      close_source(r);
      r->win.reset();
      r->pos = r->end = r->scan = 0;
      r->file_idx = r->order.size();
      return NT_OK;
    }
    off = a - r->fbase[f];
  } else {  // record b of file a
    f = a;
    skip = b;
    if (f >= r->files.size()) return NT_E_ARG;
  }
  const bool here = r->active && r->cur_file == f;
  if (mode == 0 && here && r->win && r->win->map && off <= r->end) {
    // the mapped file is open: move within it
  } else if (mode == 1 && here && r->rec_in_file <= skip) {
    skip -= r->rec_in_file;  // forward in the open file
  } else {
    size_t at = r->file_idx;
    while (at < r->order.size() && r->order[at] != f) ++at;
    if (at >= r->order.size()) {
      r->err = "seek to a file outside the reader's plan: " + r->files[f];
      return NT_E_ARG;
    }
    r->file_idx = at;
    if (!open_next(r)) return NT_E_ARG;
  }
  if (mode == 0) {
    if (off > r->end) return NT_E_ARG;
    if (r->fq_mode == 1 && r->fq_i < r->fq.size() && off >= r->fq[r->fq_i].hdr && off < r->fq_scan) {
      // a forward seek inside the indexed slice: keep the index, move to the
      // record that starts there (the records are in file order)
      size_t lo = r->fq_i, hi = r->fq.size();
      while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        if (r->fq[mid].hdr < off) lo = mid + 1;
        else hi = mid;
      }
      if (lo < r->fq.size() && r->fq[lo].hdr == off) {
        r->fq_i = lo;
        r->pos = off;
        return NT_OK;
      }
    }
    r->pos = r->scan = off;
    r->nl.clear();
    r->nl_i = 0;
    fq_reset(r, off, r->win && r->win->map != nullptr, kSliceSeek);
    return NT_OK;
  }
  std::vector<uint64_t> lens;
  while (skip > 0) {
    lens.clear();
    const int64_t k = read_records(r, std::min<uint64_t>(skip, 1u << 16), true, &lens);
    if (k <= 0 || r->cur_file != f) {
      if (r->err.empty()) r->err = "seek past the end of " + r->files[f];
      return NT_E_ARG;
    }
    skip -= (uint64_t)k;
  }
  return NT_OK;
}

int nt_reader_stats(const nt_reader* r, uint64_t* out2) {
  if (!r || !out2) return NT_E_ARG;
  out2[0] = r->bytes_parsed;
  out2[1] = r->bytes_inflated;
  return NT_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// reads/<serial>.fasta.gz: writeXStringSet(current_seq,
// output_telo_fasta, compress = TRUE) per telomeric read (NanoTel.R:1869-1873)
// -- '>' name, the sequence in 80-column lines, gzip through R's gzfile():
// zlib deflate at level 6, raw stream (windowBits -15, memLevel 8, default
// strategy), header with mtime 0, no flags, xfl 0, OS 3 (R's gzio.h), CRC-32
// and size trailer.  The files are independent: a pool of host threads, one
// text buffer, output buffer and deflate stream each (deflateReset between
// files).  Level 6 on 2-bit-entropy text runs ~8-15 MB/s a core (zlib's lazy
// matcher walks long hash chains on a 4-letter alphabet), so the writes are
// bound by compression, not by formatting or the file system.
namespace {

struct RcTable {
  uint8_t t[256];
  RcTable() {
    for (int i = 0; i < 256; ++i) t[i] = (uint8_t)i;
    const char* a = "ACGTMRWSYKVHDBNacgtmrwsykvhdbn";
    const char* b = "TGCAKYWSRMBDHVNtgcakywsrmbdhvn";
    for (int i = 0; a[i]; ++i) t[(uint8_t)a[i]] = (uint8_t)b[i];
  }
};
const RcTable kRcTable;  // Biostrings' complement of the DNA_ALPHABET letters; others kept

struct GzWriter {
  z_stream zs{};
  int level = -1;
  std::vector<uint8_t> text, out;
  ~GzWriter() {
    if (level >= 0) deflateEnd(&zs);
  }
  // the FASTA record of one read, compressed, written to path
  bool write(const char* path, const char* name, uint64_t nl, const char* seq, uint64_t sl, bool rc, int lvl) {
    const uint64_t lines = (sl + 79) / 80;
    text.resize(1 + nl + 1 + sl + lines);
    uint8_t* p = text.data();
    *p++ = '>';
    std::memcpy(p, name, nl);
    p += nl;
    *p++ = '\n';
    for (uint64_t i = 0; i < sl; i += 80) {
      const uint64_t k = std::min<uint64_t>(80, sl - i);
      if (!rc) {
        std::memcpy(p, seq + i, k);
      } else {  // reverseComplement: position i of the written read is sl - 1 - i of the input
        for (uint64_t j = 0; j < k; ++j) p[j] = kRcTable.t[(uint8_t)seq[sl - 1 - (i + j)]];
      }
      p += k;
      *p++ = '\n';
    }
    const uint64_t tn = (uint64_t)(p - text.data());
    if (level != lvl) {
      if (level >= 0) deflateEnd(&zs);
      zs = z_stream{};
      if (deflateInit2(&zs, lvl, Z_DEFLATED, -MAX_WBITS, 8, Z_DEFAULT_STRATEGY) != Z_OK) {
        level = -1;
        return false;
      }
      level = lvl;
    } else if (deflateReset(&zs) != Z_OK) {
      return false;
    }
    out.resize(10 + deflateBound(&zs, (uLong)tn) + 8);
    static const uint8_t kHead[10] = {0x1f, 0x8b, Z_DEFLATED, 0, 0, 0, 0, 0, 0, 3};
    std::memcpy(out.data(), kHead, 10);
    zs.next_in = text.data();
    zs.avail_in = (uInt)tn;
    zs.next_out = out.data() + 10;
    zs.avail_out = (uInt)(out.size() - 18);
    if (deflate(&zs, Z_FINISH) != Z_STREAM_END) return false;
    uint64_t n = 10 + zs.total_out;
    const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), text.data(), (uInt)tn);
    const uint32_t isz = (uint32_t)tn;
    for (int b = 0; b < 4; ++b) out[n + b] = (uint8_t)(crc >> (8 * b));
    for (int b = 0; b < 4; ++b) out[n + 4 + b] = (uint8_t)(isz >> (8 * b));
    n += 8;
    const int fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);
    if (fd < 0) return false;
    uint64_t w = 0;
    while (w < n) {
      const ssize_t k = ::write(fd, out.data() + w, n - w);
      if (k <= 0) {
        ::close(fd);
        return false;
      }
      w += (uint64_t)k;
    }
    return ::close(fd) == 0;
  }
};

}  // namespace

extern "C" {

int nt_write_fasta_gz(const char* const* paths, const char* const* names, const uint64_t* name_lens,
                      const char* const* seqs, const uint64_t* seq_lens, const uint8_t* rc, uint64_t n,
                      int32_t level, int32_t threads, uint64_t* err_index) {
  if (n == 0) return NT_OK;
  if (!paths || !names || !name_lens || !seqs || !seq_lens || level < 0 || level > 9) return NT_E_ARG;
  for (uint64_t i = 0; i < n; ++i)  // (one deflate call a file: its text fits a uInt)
    if (seq_lens[i] + seq_lens[i] / 80 + name_lens[i] + 3 >= (1ull << 32)) {
      if (err_index) *err_index = i;
      return NT_E_LIMIT;
    }
  unsigned nt = threads > 0 ? (unsigned)threads : host_threads();
  nt = (unsigned)std::min<uint64_t>(nt, n);
  std::atomic<uint64_t> next{0}, bad{~0ull};
  par(nt, [&](unsigned) {
    GzWriter g;
    for (uint64_t i = next++; i < n; i = next++) {
      if (!g.write(paths[i], names[i], name_lens[i], seqs[i], seq_lens[i], rc && rc[i], level)) {
        uint64_t b = bad.load();
        while (i < b && !bad.compare_exchange_weak(b, i)) {
        }
      }
    }
  });
  if (bad.load() != ~0ull) {
    if (err_index) *err_index = bad.load();
    return NT_E_IO;
  }
  return NT_OK;
}

}  // extern "C"
