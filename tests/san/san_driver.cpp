// san_driver.cpp -- the host code that parses untrusted input and packs it,
// built with AddressSanitizer + UndefinedBehaviorSanitizer (tests/san/Makefile,
// run by tests/test_sanitizers.py): the FASTA/FASTQ(.gz) reader (nt_io.cpp),
// the 2-bit packer with --rc and IUPAC exceptions,
// serials / row columns (nt_pack.cpp) and the CPU oracle
// (oracle/nanotel_oracle.c, test infrastructure).  Every check is against an
// independent plain restatement; any sanitizer report aborts the run.
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "nanotel.h"
extern "C" {
#include "nanotel_oracle.h"
}

static int g_fail = 0;
#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                           \
    }                                                                     \
  } while (0)

struct Rec {
  std::string name, seq;
};

static std::string rand_seq(std::mt19937_64& g, size_t n, const char* alpha) {
  std::string s(n, 'A');
  const size_t k = std::strlen(alpha);
  for (auto& c : s) c = alpha[g() % k];
  return s;
}

static void write_file(const std::string& path, const std::string& data, bool gz) {
  if (gz) {
    gzFile f = gzopen(path.c_str(), "wb");
    gzwrite(f, data.data(), (unsigned)data.size());
    gzclose(f);
  } else {
    FILE* f = std::fopen(path.c_str(), "wb");
    std::fwrite(data.data(), 1, data.size(), f);
    std::fclose(f);
  }
}

// FASTA with wrapping, blank / ';' lines and CRLF; FASTQ with wrapped qualities
static std::string render(const std::vector<Rec>& recs, bool fastq, std::mt19937_64& g) {
  std::string out;
  for (const auto& r : recs) {
    const char* nl = (g() % 4 == 0) ? "\r\n" : "\n";
    if (!fastq) {
      out += ">" + r.name + nl;
      const size_t w = 1 + g() % 90;
      for (size_t i = 0; i < r.seq.size(); i += w) {
        out += r.seq.substr(i, w) + nl;
        if (g() % 13 == 0) out += nl;
        if (g() % 17 == 0) out += std::string(";comment") + nl;
      }
    } else {
      out += "@" + r.name + nl + r.seq + nl + "+" + nl;
      const std::string q(r.seq.size(), 'I');
      const size_t w = g() % 3 == 0 ? std::max<size_t>(1, r.seq.size() / 3) : r.seq.size();
      for (size_t i = 0; i < q.size(); i += w) out += q.substr(i, w) + nl;
      if (q.empty()) out += nl;
    }
  }
  return out;
}

static void test_reader(std::mt19937_64& g, const std::string& dir) {
  for (int fastq = 0; fastq < 2; ++fastq)
    for (int gz = 0; gz < 2; ++gz) {
      std::vector<Rec> recs;
      for (int i = 0; i < 300; ++i)
        recs.push_back({"read " + std::to_string(i) + " x=y", rand_seq(g, fastq ? 1 + g() % 5000 : g() % 5000, "ACGTNacgtRY")});
      const std::string path = dir + "/in_" + std::to_string(fastq) + std::to_string(gz) + (fastq ? ".fq" : ".fa");
      write_file(path, render(recs, fastq, g), gz);
      nt_reader* r = nullptr;
      CHECK(nt_reader_open(path.c_str(), fastq, &r) == 0);
      CHECK(nt_reader_keep(r, 4) == 0);
      size_t k = 0, step = 0;
      for (;;) {
        const uint64_t nrec = 1 + g() % 37;
        if (step++ % 3 == 2) {
          const uint64_t* sl = nullptr;
          const int64_t n = nt_reader_skip(r, nrec, &sl);
          CHECK(n >= 0);
          if (n <= 0) break;
          for (int64_t i = 0; i < n; ++i) CHECK(sl[i] == recs[k + i].seq.size());
          k += (size_t)n;
          continue;
        }
        const char* const* names;
        const uint64_t* nl;
        const char* const* seqs;
        const uint64_t* sl;
        const int64_t n = nt_reader_next(r, nrec, &names, &nl, &seqs, &sl);
        CHECK(n >= 0);
        if (n <= 0) break;
        for (int64_t i = 0; i < n; ++i) {
          CHECK(std::string(names[i], nl[i]) == recs[k + i].name);
          CHECK(std::string(seqs[i], sl[i]) == recs[k + i].seq);
        }
        k += (size_t)n;
      }
      CHECK(k == recs.size());
      nt_reader_close(r);
    }
  // malformed FASTQ, a truncated gzip stream, an empty file
  write_file(dir + "/bad.fq", "@a\nACGT\n+\nIIII\nXX\n", false);
  write_file(dir + "/empty.fa", "", false);
  for (const char* p : {"/bad.fq", "/empty.fa"}) {
    nt_reader* r = nullptr;
    CHECK(nt_reader_open((dir + p).c_str(), std::strstr(p, ".fq") ? 1 : 0, &r) == 0);
    const char* const* names;
    const uint64_t* nl;
    const char* const* seqs;
    const uint64_t* sl;
    int64_t n = 0, tot = 0;
    while ((n = nt_reader_next(r, 2, &names, &nl, &seqs, &sl)) > 0) tot += n;
    if (std::strstr(p, "bad")) CHECK(n < 0 && std::strlen(nt_reader_error(r)) > 0);
    else CHECK(n == 0 && tot == 0);
    nt_reader_close(r);
  }
  {
    std::string big = render({{"r", rand_seq(g, 200000, "ACGT")}}, true, g);
    gzFile f = gzopen((dir + "/trunc.fq.gz").c_str(), "wb");
    gzwrite(f, big.data(), (unsigned)big.size());
    gzclose(f);
    FILE* x = std::fopen((dir + "/trunc.fq.gz").c_str(), "rb+");
    std::fseek(x, 0, SEEK_END);
    const long sz = std::ftell(x);
    std::fclose(x);
    CHECK(truncate((dir + "/trunc.fq.gz").c_str(), sz / 2) == 0);
    nt_reader* r = nullptr;
    CHECK(nt_reader_open((dir + "/trunc.fq.gz").c_str(), 1, &r) == 0);
    const char* const* names;
    const uint64_t* nl;
    const char* const* seqs;
    const uint64_t* sl;
    CHECK(nt_reader_next(r, 5, &names, &nl, &seqs, &sl) < 0);
    nt_reader_close(r);
  }
}

static int code2(char c) {
  switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
  }
  return -1;
}

static void test_packer(std::mt19937_64& g) {
  std::vector<std::string> seqs;
  for (int i = 0; i < 200; ++i) seqs.push_back(rand_seq(g, 1 + g() % 7000, i % 5 ? "ACGTacgt" : "ACGTNRYKMacgtn"));
  std::vector<const char*> ptr;
  std::vector<uint64_t> lens;
  for (auto& s : seqs) {
    ptr.push_back(s.data());
    lens.push_back(s.size());
  }
  const uint64_t n = seqs.size();
  uint64_t tb = 0, tw = 0, te = 0, ml = 0, bad = 0;
  CHECK(nt_pack_count(ptr.data(), lens.data(), n, 100, &tb, &tw, &te, &ml, &bad) == 0);
  for (int rc = 0; rc < 2; ++rc) {
    std::vector<uint32_t> planes(2 * tb + 2), len(n), eoff(n + 1), epos(te + 1);
    std::vector<uint64_t> blk(n), woff(n);
    std::vector<uint8_t> ecode(te + 1);
    CHECK(nt_pack_reads(ptr.data(), lens.data(), n, rc, 100, planes.data(), blk.data(), len.data(), woff.data(),
                        eoff.data(), epos.data(), ecode.data()) == 0);
    for (uint64_t r = 0; r < n; ++r)
      for (uint64_t p = 0; p < lens[r]; ++p) {
        const char ch = rc ? seqs[r][lens[r] - 1 - p] : seqs[r][p];
        int c = code2(ch);
        if (c < 0) c = 0;
        else if (rc) c = 3 - c;
        const uint64_t w = 2 * (blk[r] + p / 32);
        const int got = (int)((planes[w] >> (p % 32)) & 1u) | (int)(((planes[w + 1] >> (p % 32)) & 1u) << 1);
        CHECK(got == c);
      }
  }
}

static void test_serials_rows(std::mt19937_64& g) {
  for (int t = 0; t < 50; ++t) {
    const uint64_t n = g() % 40;
    std::vector<uint8_t> telo(n);
    for (auto& x : telo) x = (uint8_t)(g() % 3 == 0);
    double ss = 1.0 + (double)(g() % 5), mx = -INFINITY, ss2 = ss, mx2 = mx;
    std::vector<double> ser(n + 1), ser2(n + 1);
    std::vector<int64_t> ord(n + 1), ord2(n + 1);
    const int64_t rows = nt_assign_serials(telo.data(), n, &ss, &mx, ser.data(), ord.data());
    const int64_t rows2 = nto_assign_serials(telo.data(), (int64_t)n, &ss2, &mx2, ser2.data(), ord2.data());
    CHECK(rows == rows2 && ss == ss2 && mx == mx2);
    for (int64_t i = 0; i < rows; ++i) CHECK(ord[i] == ord2[i]);
    std::vector<int32_t> st(3 * n + 3), en(3 * n + 3);
    std::vector<double> de(3 * n + 3);
    std::vector<uint64_t> ln(n + 1);
    for (uint64_t i = 0; i < 3 * n; ++i) {
      st[i] = g() % 4 == 0 ? -1 : (int32_t)(g() % 1000);
      en[i] = st[i] + (int32_t)(g() % 100);
      de[i] = (double)(g() % 100) / 100.0;
    }
    for (uint64_t i = 0; i < n; ++i) ln[i] = 1 + g() % 100000;
    const int64_t r = rows > 0 ? rows : 1;
    std::vector<double> cs(r), cd(3 * r);
    std::vector<int32_t> cl(r), c1(3 * r), c2(3 * r), c3(3 * r);
    CHECK(nt_rows_columns(st.data(), en.data(), de.data(), ln.data(), n, 3, ser.data(), ord.data(), rows, cs.data(),
                          cl.data(), cd.data(), c1.data(), c2.data(), c3.data()) == rows);
    for (int64_t i = 0; i < rows; ++i)
      for (int p = 0; p < 3; ++p) {
        const int64_t j = ord[i];
        if (st[3 * j + p] == -1) CHECK(c1[p * rows + i] == NT_NA_INT32 && std::isnan(cd[p * rows + i]));
        else CHECK(c3[p * rows + i] == en[3 * j + p] - st[3 * j + p] + 1);
      }
  }
}

static void test_oracle(std::mt19937_64& g) {
  const char* cfg[][2] = {{"TTAGGG", nullptr}, {"YYAGGG", nullptr}, {"TTAGGG TCAGGG", "TGAGGG TTGGGG"},
                          {"TAGGGTTAGGGTTAGGGT", nullptr}, {"TTAGGN CCCTAA", "TTAGGGTTAGGGTTAGGGTTAGGGTTAGGGTTAGG"}};
  for (auto& c : cfg) {
    int err = 0;
    nto_patterns* P = nto_patterns_new(c[0], c[1], &err);
    CHECK(P != nullptr);
    if (!P) continue;
    for (int i = 0; i < 40; ++i) {
      std::string s = rand_seq(g, 1 + g() % 6000, i % 4 ? "ACGT" : "ACGTNRY");
      const size_t tl = std::min<size_t>(s.size(), g() % 3000);
      for (size_t p = 0; p < tl; ++p) s[p] = "TTAGGG"[p % 6];
      nto_row row;
      const int64_t nw = nto_window_count((int64_t)s.size(), 100);
      std::vector<uint32_t> wc(3 * (nw + 1)), hits(64);
      const int rc = nto_analyze_read(s.data(), (int64_t)s.size(), P, 100, 0.6, i % 7 == 0 && s.size() > 50,
                                      0, &row, wc.data(), hits.data());
      CHECK(rc == 0);
    }
    nto_patterns_free(P);
  }
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  std::mt19937_64 g(20261017);
  test_reader(g, argv[1]);
  test_packer(g);
  test_serials_rows(g);
  test_oracle(g);
  std::printf("san_driver: %s (%d failed checks)\n", g_fail ? "FAIL" : "OK", g_fail);
  return g_fail ? 1 : 0;
}
