// nt_io.cpp -- streaming FASTA/FASTQ(.gz) reader in nrec-record chunks
// (SURVEY §8(f) row 1): the host ingest of run_future_worker_chuncks
// (NanoTel.R:2171-2216), i.e. XVector's open_input_files + readDNAStringSet(
// files, nrec = nrec, format = format).
//
//  * input_path is a file, or a directory whose files are listed recursively
//    and sorted by full path (dir(full.names = TRUE, recursive = TRUE),
//    NanoTel.R:2176-2178); the files form ONE record stream, a chunk may span
//    files;
//  * gzip is transparent (zlib gzread also reads plain files);
//  * FASTA: '>' starts a record whose name is the rest of the header line;
//    sequence lines are concatenated (line breaks and '\r' dropped, blank
//    lines skipped); FASTQ: 4-line records '@name', sequence, '+...', quality
//    (quality dropped);
//  * letters are kept as they are: validation against DNA_ALPHABET happens in
//    nt_pack_count (NT_E_LETTER), as readDNAStringSet would fail.
#include <dirent.h>
#include <sys/stat.h>
#include <zlib.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "nanotel.h"

struct nt_reader {
  std::vector<std::string> files;
  size_t file_idx = 0;
  gzFile gz = nullptr;
  int format = 0;  // 0 fasta, 1 fastq
  std::vector<char> buf;
  size_t pos = 0, end = 0;
  bool eof_file = true;
  std::string err;
  std::string pending_header;  // FASTA: header already read for the next record
  bool has_pending = false;
  // current chunk storage
  std::string names_blob, seqs_blob;
  std::vector<uint64_t> name_off, seq_off;
  std::vector<const char*> name_ptr, seq_ptr;
  std::vector<uint64_t> name_len, seq_len;
  uint64_t records_total = 0;
};

namespace {

void list_files(const std::string& path, std::vector<std::string>& out) {
  DIR* d = opendir(path.c_str());
  if (!d) return;
  while (dirent* e = readdir(d)) {
    const std::string n = e->d_name;
    if (n == "." || n == "..") continue;
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
  if (r->file_idx >= r->files.size()) return false;
  r->gz = gzopen(r->files[r->file_idx++].c_str(), "rb");
  if (!r->gz) {
    r->err = "cannot open " + r->files[r->file_idx - 1];
    return false;
  }
  gzbuffer(r->gz, 1 << 20);
  r->pos = r->end = 0;
  r->eof_file = false;
  return true;
}

// One line of the current file (without '\n' / '\r'); false at end of file.
bool get_line(nt_reader* r, std::string& line) {
  line.clear();
  if (!r->gz) return false;
  for (;;) {
    if (r->pos == r->end) {
      if (r->eof_file) return !line.empty();
      const int n = gzread(r->gz, r->buf.data(), (unsigned)r->buf.size());
      if (n <= 0) {
        r->eof_file = true;
        return !line.empty();
      }
      r->pos = 0;
      r->end = (size_t)n;
    }
    const char* b = r->buf.data() + r->pos;
    const char* nl = (const char*)memchr(b, '\n', r->end - r->pos);
    if (nl) {
      line.append(b, nl - b);
      r->pos += (nl - b) + 1;
      if (!line.empty() && line.back() == '\r') line.pop_back();
      return true;
    }
    line.append(b, r->end - r->pos);
    r->pos = r->end;
  }
}

void add_record(nt_reader* r, const std::string& name, const std::string& seq) {
  r->name_off.push_back(r->names_blob.size());
  r->name_len.push_back(name.size());
  r->names_blob += name;
  r->seq_off.push_back(r->seqs_blob.size());
  r->seq_len.push_back(seq.size());
  r->seqs_blob += seq;
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
    std::string plus, qual;
    if (!get_line(r, seq) || !get_line(r, plus) || plus.empty() || plus[0] != '+') {
      r->err = "malformed FASTQ record '" + name + "'";
      return false;
    }
    // quality may in principle wrap; consume lines until its length matches
    size_t ql = 0;
    while (ql < seq.size() && get_line(r, qual)) ql += qual.size();
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
  r->names_blob.clear();
  r->seqs_blob.clear();
  r->name_off.clear();
  r->seq_off.clear();
  r->name_len.clear();
  r->seq_len.clear();
  if (!r->gz && r->file_idx == 0 && !open_next(r)) return r->err.empty() ? 0 : NT_E_ARG;
  std::string name, seq;
  while (r->name_len.size() < nrec) {
    if (!next_record(r, name, seq)) {
      if (!r->err.empty()) return NT_E_ARG;
      break;
    }
    add_record(r, name, seq);
  }
  const size_t n = r->name_len.size();
  r->name_ptr.resize(n);
  r->seq_ptr.resize(n);
  for (size_t i = 0; i < n; ++i) {
    r->name_ptr[i] = r->names_blob.data() + r->name_off[i];
    r->seq_ptr[i] = r->seqs_blob.data() + r->seq_off[i];
  }
  *names = r->name_ptr.data();
  *name_lens = r->name_len.data();
  *seqs = r->seq_ptr.data();
  *seq_lens = r->seq_len.data();
  r->records_total += n;
  return (int64_t)n;
}

}  // extern "C"
