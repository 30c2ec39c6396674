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
#include <sys/stat.h>
#include <zlib.h>

#include <algorithm>
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
    bool done = false;
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
      gzFile g = gzopen((*files)[i].c_str(), "rb");
      if (!g) {
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
  bool take(size_t i, std::vector<char>& out, std::string& err) {
    std::unique_lock<std::mutex> lk(mu);
    consumed = i + 1;
    cv.notify_all();
    cv.wait(lk, [&] { return slots[i].done; });
    if (!slots[i].err.empty()) {
      err = slots[i].err;
      return false;
    }
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
  size_t file_idx = 0;
  gzFile gz = nullptr;
  bool active = false;  // a file is open (streamed through gz, or inflated in buf)
  std::unique_ptr<Prefetcher> pf;
  int format = 0;  // 0 fasta, 1 fastq
  std::vector<char> buf;
  size_t pos = 0, end = 0;
  bool eof_file = true;
  std::string err;
  std::string pending_header;  // FASTA: header already read for the next record
  bool has_pending = false;
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
  bool seq_direct = false;  // FASTQ: next_record wrote the sequence into seqs_blob at seq_mark
  size_t seq_mark = 0;
  uint64_t records_total = 0;
};

namespace {

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

bool open_next(nt_reader* r) {
  if (r->gz) {
    gzclose(r->gz);
    r->gz = nullptr;
  }
  r->active = false;
  if (!r->err.empty() || r->file_idx >= r->files.size()) return false;
  if (r->pf) {  // inflated ahead by the workers: parse straight from memory
    if (!r->pf->take(r->file_idx++, r->buf, r->err)) return false;
    r->pos = 0;
    r->end = r->buf.size();
    r->eof_file = true;
    r->active = true;
    return true;
  }
  r->gz = gzopen(r->files[r->file_idx++].c_str(), "rb");
  if (!r->gz) {
    r->err = "cannot open " + r->files[r->file_idx - 1];
    return false;
  }
  gzbuffer(r->gz, 1 << 20);
  if (r->buf.size() != (1u << 20)) std::vector<char>(1 << 20).swap(r->buf);
  r->pos = r->end = 0;
  r->eof_file = false;
  r->active = true;
  return true;
}

// One line of the current file (without '\n' / '\r') appended to `out`
// (nullptr: skipped, e.g. FASTQ qualities); false at end of file.  Returns the
// line length through `len`.
bool take_line(nt_reader* r, std::string* out, size_t* len = nullptr) {
  if (!r->active) return false;
  const size_t base = out ? out->size() : 0;
  size_t n_line = 0;
  bool any = false;
  for (;;) {
    if (r->pos == r->end) {
      if (r->eof_file) break;
      const int n = gzread(r->gz, r->buf.data(), (unsigned)r->buf.size());
      if (n < 0 || (n == 0 && gz_failed(r->gz)))  // corrupt or truncated gzip stream
        r->err = "read error in " + r->files[r->file_idx - 1];
      if (n <= 0) {
        r->eof_file = true;
        break;
      }
      r->pos = 0;
      r->end = (size_t)n;
    }
    any = true;
    const char* b = r->buf.data() + r->pos;
    const char* nl = (const char*)memchr(b, '\n', r->end - r->pos);
    const size_t k = nl ? (size_t)(nl - b) : r->end - r->pos;
    if (out) out->append(b, k);
    n_line += k;
    r->pos += k;
    if (nl) {
      ++r->pos;
      if (out && out->size() > base && out->back() == '\r') out->pop_back(), --n_line;
      else if (!out && k && b[k - 1] == '\r') --n_line;
      if (len) *len = n_line;
      return true;
    }
  }
  if (len) *len = n_line;
  return any && n_line > 0;
}

bool get_line(nt_reader* r, std::string& line) {
  line.clear();
  return take_line(r, &line);
}

void add_record(nt_reader* r, const std::string& name, const std::string& seq) {
  r->c().name_off.push_back(r->c().names_blob.size());
  r->c().name_len.push_back(name.size());
  r->c().names_blob += name;
  if (r->seq_direct) {  // FASTQ: already in the blob from seq_mark on
    r->c().seq_len.push_back(r->c().seqs_blob.size() - r->seq_mark);
  } else {
    r->c().seq_off.push_back(r->c().seqs_blob.size());
    r->c().seq_len.push_back(seq.size());
    r->c().seqs_blob += seq;
    return;
  }
  r->c().seq_off.push_back(r->seq_mark);
}

// Next record of the stream; false at the end of all files (or error).
bool next_record(nt_reader* r, std::string& name, std::string& seq) {
  std::string line;
  seq.clear();
  for (;;) {
    if (r->format == 0) {
      if (!r->has_pending) {
        // find the next header
        bool got = false;
        while (get_line(r, line)) {
          if (!line.empty() && line[0] == '>') {
            r->pending_header = line.substr(1);
            r->has_pending = got = true;
            break;
          }
        }
        if (!got) {
          if (!open_next(r)) return false;
          continue;
        }
      }
      name = r->pending_header;
      r->has_pending = false;
      while (get_line(r, line)) {
        if (line.empty() || line[0] == ';') continue;
        if (line[0] == '>') {
          r->pending_header = line.substr(1);
          r->has_pending = true;
          break;
        }
        seq += line;
      }
      return true;
    }
    // FASTQ
    bool got = false;
    while (get_line(r, line)) {
      if (line.empty()) continue;
      if (line[0] != '@') {
        r->err = "malformed FASTQ record (expected '@')";
        return false;
      }
      got = true;
      break;
    }
    if (!got) {
      if (!open_next(r)) return false;
      continue;
    }
    name = line.substr(1);
    // the sequence line goes straight into the chunk's blob (seq_direct)
    std::string plus;
    const size_t s0 = r->c().seqs_blob.size();
    size_t sl = 0, ql = 0, k = 0;
    if (!take_line(r, &r->c().seqs_blob, &sl) || !get_line(r, plus) || plus.empty() || plus[0] != '+') {
      r->c().seqs_blob.resize(s0);
      r->err = "malformed FASTQ record '" + name + "'";
      return false;
    }
    // quality may in principle wrap; skip lines until its length matches
    while (ql < sl && take_line(r, nullptr, &k)) ql += k;
    r->seq_mark = s0;
    r->seq_direct = true;
    return true;
  }
}

// First byte of the current file's next line (refilling the buffer), -1 at
// the end of the file.
int peek_byte(nt_reader* r) {
  if (!r->active) return -1;
  if (r->pos == r->end) {
    if (r->eof_file) return -1;
    const int n = gzread(r->gz, r->buf.data(), (unsigned)r->buf.size());
    if (n < 0 || (n == 0 && gz_failed(r->gz))) r->err = "read error in " + r->files[r->file_idx - 1];
    if (n <= 0) {
      r->eof_file = true;
      return -1;
    }
    r->pos = 0;
    r->end = (size_t)n;
  }
  return (unsigned char)r->buf[r->pos];
}

// next_record without the copies: the record's sequence length only (the
// same parse and the same errors; names are short and parsed into a scratch
// string).  false at the end of all files (or error).
bool skip_record(nt_reader* r, uint64_t& len) {
  std::string line;
  len = 0;
  for (;;) {
    if (r->format == 0) {
      if (!r->has_pending) {
        bool got = false;
        while (get_line(r, line)) {
          if (!line.empty() && line[0] == '>') {
            r->pending_header = line.substr(1);
            r->has_pending = got = true;
            break;
          }
        }
        if (!got) {
          if (!open_next(r)) return false;
          continue;
        }
      }
      r->has_pending = false;
      for (;;) {
        const int c = peek_byte(r);
        if (c < 0) break;
        if (c == '>') {  // the next record's header (its name is needed if next_record reads it)
          get_line(r, line);
          r->pending_header = line.substr(1);
          r->has_pending = true;
          break;
        }
        size_t k = 0;
        if (!take_line(r, nullptr, &k)) break;
        if (c != ';') len += k;  // ';' comment lines are dropped, as next_record does
      }
      return true;
    }
    bool got = false;
    while (get_line(r, line)) {
      if (line.empty()) continue;
      if (line[0] != '@') {
        r->err = "malformed FASTQ record (expected '@')";
        return false;
      }
      got = true;
      break;
    }
    if (!got) {
      if (!open_next(r)) return false;
      continue;
    }
    const std::string name = line.substr(1);
    std::string plus;
    size_t sl = 0, ql = 0, k = 0;
    if (!take_line(r, nullptr, &sl) || !get_line(r, plus) || plus.empty() || plus[0] != '+') {
      r->err = "malformed FASTQ record '" + name + "'";
      return false;
    }
    while (ql < sl && take_line(r, nullptr, &k)) ql += k;
    len = sl;
    return true;
  }
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
  r->buf.resize(1 << 20);
  if (r->files.size() > 1) {  // a run directory: inflate parts ahead on worker threads
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
  if (r->gz) gzclose(r->gz);
  delete r;
}

uint64_t nt_reader_file_count(const nt_reader* r) { return r ? r->files.size() : 0; }

const char* nt_reader_file(const nt_reader* r, uint64_t i) {
  return (r && i < r->files.size()) ? r->files[i].c_str() : nullptr;
}

const char* nt_reader_error(const nt_reader* r) { return r ? r->err.c_str() : "null reader"; }

int64_t nt_reader_next(nt_reader* r, uint64_t nrec, const char* const** names,
                       const uint64_t** name_lens, const char* const** seqs,
                       const uint64_t** seq_lens) {
  if (!r || !names || !name_lens || !seqs || !seq_lens || nrec == 0) return NT_E_ARG;
  r->cur ^= 1;
  r->c().names_blob.clear();
  r->c().seqs_blob.clear();
  r->c().name_off.clear();
  r->c().seq_off.clear();
  r->c().name_len.clear();
  r->c().seq_len.clear();
  if (!r->active && r->file_idx == 0 && !open_next(r)) return r->err.empty() ? 0 : NT_E_ARG;
  std::string name, seq;
  while (r->c().name_len.size() < nrec) {
    r->seq_direct = false;
    if (!next_record(r, name, seq)) {
      if (!r->err.empty()) return NT_E_ARG;
      break;
    }
    add_record(r, name, seq);
  }
  const size_t n = r->c().name_len.size();
  r->c().name_ptr.resize(n);
  r->c().seq_ptr.resize(n);
  for (size_t i = 0; i < n; ++i) {
    r->c().name_ptr[i] = r->c().names_blob.data() + r->c().name_off[i];
    r->c().seq_ptr[i] = r->c().seqs_blob.data() + r->c().seq_off[i];
  }
  *names = r->c().name_ptr.data();
  *name_lens = r->c().name_len.data();
  *seqs = r->c().seq_ptr.data();
  *seq_lens = r->c().seq_len.data();
  r->records_total += n;
  return (int64_t)n;
}

int64_t nt_reader_skip(nt_reader* r, uint64_t nrec, const uint64_t** seq_lens) {
  if (!r || !seq_lens || nrec == 0) return NT_E_ARG;
  r->cur ^= 1;
  r->c().names_blob.clear();
  r->c().seqs_blob.clear();
  r->c().name_off.clear();
  r->c().seq_off.clear();
  r->c().name_len.clear();
  r->c().seq_len.clear();
  r->c().name_ptr.clear();
  r->c().seq_ptr.clear();
  if (!r->active && r->file_idx == 0 && !open_next(r)) return r->err.empty() ? 0 : NT_E_ARG;
  uint64_t len = 0;
  while (r->c().seq_len.size() < nrec) {
    if (!skip_record(r, len)) {
      if (!r->err.empty()) return NT_E_ARG;
      break;
    }
    r->c().seq_len.push_back(len);
  }
  const size_t n = r->c().seq_len.size();
  *seq_lens = r->c().seq_len.data();
  r->records_total += n;
  return (int64_t)n;
}

}  // extern "C"
