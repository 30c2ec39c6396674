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

// Whole-file inflation of the next files of a multi-file input, ahead of the
// parser: worker threads take files in order, at most `window` beyond the one
// being parsed; the parser waits for its file's buffer.
struct Prefetcher {
  struct Slot {
    bool done = false, plain = false;  // plain: not gzip, the parser reads it itself (parallel pread)
    std::string err;
    std::vector<char> data;
  };
  const std::vector<std::string>* files = nullptr;
  std::vector<Slot> slots;
  size_t next = 0, consumed = 0, window = 1;
  bool stop = false;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::thread> workers;

  void start(const std::vector<std::string>& f, unsigned n_threads) {
    files = &f;
    slots.resize(f.size());
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
        for (;;) {
          if (sl.data.size() - used < (4u << 20)) sl.data.resize(std::max<size_t>(8u << 20, sl.data.size() * 2));
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
  bool take(size_t i, std::vector<char>& out, bool& plain, std::string& err) {
    std::unique_lock<std::mutex> lk(mu);
    consumed = i + 1;
    cv.notify_all();
    cv.wait(lk, [&] { return slots[i].done; });
    if (!slots[i].err.empty()) {
      err = slots[i].err;
      return false;
    }
    plain = slots[i].plain;
    if (plain) return true;
    out.swap(slots[i].data);
    std::vector<char>().swap(slots[i].data);
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

struct nt_reader {
  std::vector<std::string> files;
  size_t file_idx = 0;  // next file to open
  int format = 0;       // 0 fasta, 1 fastq
  // the current file's bytes come from a plain descriptor (parallel pread), a
  // gzip stream (serial inflate) or a whole file inflated ahead (Prefetcher)
  int fd = -1;
  uint64_t fsize = 0, foff = 0;
  gzFile gz = nullptr;
  bool active = false;   // a file is open
  bool src_eof = true;   // no bytes of the current file beyond buf[end)
  std::unique_ptr<Prefetcher> pf;
  // the window: bytes [pos, end) of buf not yet parsed; nl = offsets (into buf)
  // of the '\n' in [scan, end), nl[nl_i] the first one at or after pos
  std::vector<char> buf;
  size_t pos = 0, end = 0, scan = 0;
  std::vector<uint64_t> nl;
  size_t nl_i = 0;
  std::string err;
  // chunk storage, two slots used in turn: a chunk stays valid through the
  // next nt_reader_next call (so the caller can read chunk k+1 on another
  // thread while it still scans chunk k)
  struct Store {
    std::string names_blob, seqs_blob;
    std::vector<uint64_t> name_off, seq_off;
    std::vector<const char*> name_ptr, seq_ptr;
    std::vector<uint64_t> name_len, seq_len;
  } store[2];
  int cur = 0;
  Store& c() { return store[cur]; }
  // records parsed from the window and not yet copied into the chunk store:
  // name range, sequence pieces [piece0, piece1) of `pieces` (offset, length in buf)
  struct Pend {
    uint64_t name_at, name_len, piece0, piece1, seq_len;
  };
  std::vector<Pend> pend;
  std::vector<std::pair<uint64_t, uint64_t>> pieces;
  uint64_t records_total = 0;
};

namespace {

constexpr size_t kWindow0 = 64u << 20;  // window bytes (grows for a record that does not fit)

unsigned host_threads() {
  unsigned nt = std::thread::hardware_concurrency();
  nt = std::max(1u, std::min(nt == 0 ? 1u : nt, 16u));
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
  if (r->fd >= 0) ::close(r->fd);
  r->fd = -1;
  r->active = false;
}

// the '\n' offsets of buf[scan, end): parallel memchr over large ranges
void index_lines(nt_reader* r) {
  const size_t a = r->scan, b = r->end;
  if (b <= a) return;
  const char* base = r->buf.data();
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
  const unsigned nt = (b - a) >= (8u << 20) ? host_threads() : 1u;
  if (nt == 1) {
    scan_range(a, b, r->nl);
  } else {
    std::vector<std::vector<uint64_t>> part(nt);
    par(nt, [&](unsigned t) { scan_range(a + (b - a) * t / nt, a + (b - a) * (t + 1) / nt, part[t]); });
    for (auto& v : part) r->nl.insert(r->nl.end(), v.begin(), v.end());
  }
  r->scan = b;
}

// Make room and read more of the current file after buf[end): the unparsed
// bytes [pos, end) move to the front first.  Returns false when nothing more
// can come (end of the file, or an error).
bool fill(nt_reader* r) {
  if (r->src_eof || !r->active) return false;
  // move the unparsed tail (and its line index) to the front
  if (r->pos > 0) {
    const size_t keep = r->end - r->pos;
    std::memmove(r->buf.data(), r->buf.data() + r->pos, keep);
    size_t j = 0;
    for (size_t i = r->nl_i; i < r->nl.size(); ++i) r->nl[j++] = r->nl[i] - r->pos;
    r->nl.resize(j);
    r->nl_i = 0;
    r->scan -= r->pos;
    r->end = keep;
    r->pos = 0;
  }
  if (r->buf.size() < kWindow0) r->buf.resize(kWindow0);
  if (r->end * 2 > r->buf.size()) r->buf.resize(r->buf.size() * 2);  // a record larger than half the window
  const size_t room = r->buf.size() - r->end;
  if (r->fd >= 0) {  // plain file: parallel pread of the next `want` bytes
    const uint64_t want = std::min<uint64_t>(room, r->fsize - r->foff);
    const unsigned nt = want >= (8u << 20) ? host_threads() : 1u;
    std::atomic<bool> bad{false};
    char* dst = r->buf.data() + r->end;
    const uint64_t off0 = r->foff;
    par(nt, [&](unsigned t) {
      uint64_t x = want * t / nt;
      const uint64_t y = want * (t + 1) / nt;
      while (x < y) {
        const ssize_t k = ::pread(r->fd, dst + x, (size_t)(y - x), (off_t)(off0 + x));
        if (k <= 0) {
          bad = true;
          return;
        }
        x += (uint64_t)k;
      }
    });
    if (bad) {
      r->err = "read error in " + r->files[r->file_idx - 1];
      r->src_eof = true;
      return false;
    }
    r->foff += want;
    r->end += want;
    r->src_eof = r->foff >= r->fsize;
    index_lines(r);
    return want > 0;
  }
  // gzip stream: serial inflate into the room
  size_t got = 0;
  while (got < room) {
    const int n = gzread(r->gz, r->buf.data() + r->end + got, (unsigned)std::min<size_t>(room - got, 1u << 30));
    if (n < 0 || (n == 0 && gz_failed(r->gz))) {  // corrupt or truncated gzip stream
      r->err = "read error in " + r->files[r->file_idx - 1];
      r->src_eof = true;
      return false;
    }
    if (n == 0) {
      r->src_eof = true;
      break;
    }
    got += (size_t)n;
  }
  r->end += got;
  index_lines(r);
  return got > 0;
}

bool open_next(nt_reader* r) {
  close_source(r);
  r->pos = r->end = r->scan = 0;
  r->nl.clear();
  r->nl_i = 0;
  if (!r->err.empty() || r->file_idx >= r->files.size()) return false;
  const std::string& path = r->files[r->file_idx++];
  if (r->pf) {  // a gzip part inflated ahead by the workers: parse straight from memory
    bool plain = false;
    if (!r->pf->take(r->file_idx - 1, r->buf, plain, r->err)) return false;
    if (!plain) {
      r->end = r->buf.size();
      r->src_eof = true;
      r->active = true;
      index_lines(r);
      return true;
    }
  }
  if (!is_gzip(path)) {
    r->fd = ::open(path.c_str(), O_RDONLY);
    struct stat st;
    if (r->fd < 0 || fstat(r->fd, &st) != 0) {
      r->err = "cannot open " + path;
      close_source(r);
      return false;
    }
    r->fsize = (uint64_t)st.st_size;
    r->foff = 0;
  } else {
    r->gz = gzopen(path.c_str(), "rb");
    if (!r->gz) {
      r->err = "cannot open " + path;
      return false;
    }
    gzbuffer(r->gz, 1 << 20);
  }
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
// window holds no complete line there: more bytes may come (need = true), or
// the file is exhausted (need = false).  At the end of a file the last,
// unterminated line counts when it is not empty.
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
    if (!r->src_eof) {
      need = true;
      return false;
    }
    le = r->end;
    c.p = r->end;
  }
  if (le > ls && r->buf[le - 1] == '\r') --le;
  return true;
}

// One record from the window at the committed cursor; appended to r->pend
// (or, when lens_only, its sequence length to `len`).  Returns 1 = a record,
// 0 = end of this file, -1 = error, 2 = incomplete (fill and retry).
int parse_record(nt_reader* r, bool lens_only, uint64_t& len) {
  Cur c{r->pos, r->nl_i};
  size_t ls = 0, le = 0;
  bool need = false;
  const char* b = r->buf.data();
  len = 0;
  if (r->format == 0) {
    uint64_t name_at = 0, name_len = 0;
    for (;;) {  // the header (lines before the first one are skipped)
      if (!next_line(r, c, ls, le, need)) return need ? 2 : 0;
      if (le > ls && b[ls] == '>') break;
    }
    name_at = ls + 1;
    name_len = le - ls - 1;
    const size_t p0 = r->pieces.size();
    for (;;) {  // sequence lines up to the next header or the end of the file
      Cur save = c;
      if (!next_line(r, c, ls, le, need)) {
        if (need) {
          r->pieces.resize(p0);
          return 2;
        }
        break;
      }
      if (le == ls || b[ls] == ';') continue;  // blank and ';' comment lines are dropped
      if (b[ls] == '>') {
        c = save;  // the next record's header
        break;
      }
      len += le - ls;
      if (!lens_only) r->pieces.emplace_back(ls, le - ls);
    }
    r->pos = c.p;
    r->nl_i = c.i;
    if (!lens_only) r->pend.push_back({name_at, name_len, p0, r->pieces.size(), len});
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
  const uint64_t name_at = ls + 1, name_len = le - ls - 1;
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
  r->pos = c.p;
  r->nl_i = c.i;
  len = sl;
  if (!lens_only) {
    r->pieces.emplace_back(ss, sl);
    r->pend.push_back({name_at, name_len, r->pieces.size() - 1, r->pieces.size(), sl});
  }
  return 1;
}

// Copy the pending records' names and sequences into the chunk store (all
// host threads over the records), before the window moves.
void flush_pending(nt_reader* r) {
  if (r->pend.empty()) return;
  auto& S = r->c();
  const size_t n0 = S.name_len.size(), m = r->pend.size();
  uint64_t nb = S.names_blob.size(), sb = S.seqs_blob.size();
  S.name_off.resize(n0 + m);
  S.name_len.resize(n0 + m);
  S.seq_off.resize(n0 + m);
  S.seq_len.resize(n0 + m);
  for (size_t k = 0; k < m; ++k) {
    const auto& q = r->pend[k];
    S.name_off[n0 + k] = nb;
    S.name_len[n0 + k] = q.name_len;
    S.seq_off[n0 + k] = sb;
    S.seq_len[n0 + k] = q.seq_len;
    nb += q.name_len;
    sb += q.seq_len;
  }
  S.names_blob.resize(nb);
  S.seqs_blob.resize(sb);
  const char* b = r->buf.data();
  char* nd = &S.names_blob[0];
  char* sd = &S.seqs_blob[0];
  const uint64_t bytes = sb;
  const unsigned nt = (bytes >= (4u << 20) && m > 1) ? std::min<unsigned>(host_threads(), (unsigned)m) : 1u;
  par(nt, [&](unsigned t) {
    for (size_t k = m * t / nt; k < m * (t + 1) / nt; ++k) {
      const auto& q = r->pend[k];
      std::memcpy(nd + S.name_off[n0 + k], b + q.name_at, q.name_len);
      char* o = sd + S.seq_off[n0 + k];
      for (uint64_t j = q.piece0; j < q.piece1; ++j) {
        std::memcpy(o, b + r->pieces[j].first, r->pieces[j].second);
        o += r->pieces[j].second;
      }
    }
  });
  r->pend.clear();
  r->pieces.clear();
}

// Up to nrec records into the chunk store (or their lengths only); returns
// the count, or -1 on error.
int64_t read_records(nt_reader* r, uint64_t nrec, bool lens_only) {
  auto& S = r->c();
  uint64_t got = 0;
  while (got < nrec) {
    if (!r->active) {
      flush_pending(r);
      if (!open_next(r)) break;
      continue;
    }
    uint64_t len = 0;
    const int k = parse_record(r, lens_only, len);
    if (k == 1) {
      ++got;
      if (lens_only) S.seq_len.push_back(len);
      continue;
    }
    if (k < 0) return -1;
    if (k == 2) {  // incomplete: copy what is parsed, then read more of the file
      flush_pending(r);
      if (!fill(r) && !r->err.empty()) return -1;
      continue;
    }
    flush_pending(r);  // k == 0: this file is done
    if (!r->err.empty()) return -1;
    close_source(r);
  }
  flush_pending(r);
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
  if (r->files.size() > 1) {  // a run directory: inflate gzip parts ahead on worker threads
    unsigned nt = std::thread::hardware_concurrency();
    nt = std::max(1u, std::min(nt == 0 ? 1u : nt, 16u));
    if (const char* v = std::getenv("NT_READER_THREADS")) nt = (unsigned)std::max(0, atoi(v));
    if (nt > 0) {
      r->pf.reset(new Prefetcher());
      r->pf->start(r->files, nt);
    }
  }
  *out = r;
  return NT_OK;
}

void nt_reader_close(nt_reader* r) {
  if (!r) return;
  close_source(r);
  delete r;
}

uint64_t nt_reader_file_count(const nt_reader* r) { return r ? r->files.size() : 0; }

const char* nt_reader_file(const nt_reader* r, uint64_t i) {
  return (r && i < r->files.size()) ? r->files[i].c_str() : nullptr;
}

const char* nt_reader_error(const nt_reader* r) { return r ? r->err.c_str() : "null reader"; }

static void clear_store(nt_reader* r) {
  r->cur ^= 1;
  auto& S = r->c();
  S.names_blob.clear();
  S.seqs_blob.clear();
  S.name_off.clear();
  S.seq_off.clear();
  S.name_len.clear();
  S.seq_len.clear();
  S.name_ptr.clear();
  S.seq_ptr.clear();
}

int64_t nt_reader_next(nt_reader* r, uint64_t nrec, const char* const** names,
                       const uint64_t** name_lens, const char* const** seqs,
                       const uint64_t** seq_lens) {
  if (!r || !names || !name_lens || !seqs || !seq_lens || nrec == 0) return NT_E_ARG;
  clear_store(r);
  const int64_t n = read_records(r, nrec, false);
  if (n < 0) return NT_E_ARG;
  auto& S = r->c();
  S.name_ptr.resize((size_t)n);
  S.seq_ptr.resize((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    S.name_ptr[i] = S.names_blob.data() + S.name_off[i];
    S.seq_ptr[i] = S.seqs_blob.data() + S.seq_off[i];
  }
  *names = S.name_ptr.data();
  *name_lens = S.name_len.data();
  *seqs = S.seq_ptr.data();
  *seq_lens = S.seq_len.data();
  r->records_total += (uint64_t)n;
  return n;
}

int64_t nt_reader_skip(nt_reader* r, uint64_t nrec, const uint64_t** seq_lens) {
  if (!r || !seq_lens || nrec == 0) return NT_E_ARG;
  clear_store(r);
  const int64_t n = read_records(r, nrec, true);
  if (n < 0) return NT_E_ARG;
  *seq_lens = r->c().seq_len.data();
  r->records_total += (uint64_t)n;
  return n;
}

}  // extern "C"
