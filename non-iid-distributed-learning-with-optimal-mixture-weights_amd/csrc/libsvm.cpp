// LIBSVM / svmlight text reader (host).  Replaces the parse step of the reference's
// `svmlight_data` (/root/reference/functions/utils.py:36-38: sklearn's load_svmlight_file)
// for the dense float32 rows `load_full_data` feeds the feature map (utils.py:56, `.A` then
// float32): every value parsed as a double (correctly rounded, as Python's float()) and
// rounded once to float32, exactly as `csr.toarray().astype(np.float32)` rounds it.
//
// Format, as load_svmlight_file reads it: one sample per line, `label [qid:q] idx:val ...`,
// `#` starts a comment, blank / comment-only lines are skipped; the indices of a line must
// be strictly increasing (sorted and unique, else an error, as sklearn's ValueError).  Index base: zero_based = 1
// (indices start at 0), 0 (start at 1), -1 "auto" (zero-based iff the smallest index in the
// file is 0 -- sklearn's 'auto').  Width: caller's n_features (scan reports the max index).
//
// The file is read once into memory and cut into line-aligned chunks parsed by a pool of
// threads: each chunk first counts its samples (row offsets = prefix sums), then parses
// into its rows of the caller's dense matrix.
#include <algorithm>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/fedsim.h"

namespace fs {
int fail(int code, const std::string& msg);   // host.cpp
}

namespace {

struct Chunk {
  const char* b;
  const char* e;
  int64_t rows = 0;          // samples in this chunk
  int64_t first_line = 0;    // 1-based line number of the chunk's first line
  int64_t min_idx = INT64_MAX, max_idx = -1;
  std::string err;
};

bool read_file(const char* path, std::vector<char>& buf) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  buf.resize(n > 0 ? (size_t)n + 1 : 1);
  const size_t got = n > 0 ? std::fread(buf.data(), 1, (size_t)n, f) : 0;
  std::fclose(f);
  if (n > 0 && got != (size_t)n) return false;
  buf[got] = '\0';                                  // strtod / strtoll stop at the end
  buf.resize(got + 1);
  return true;
}

// line-aligned chunks of [0, n) for up to `parts` workers
std::vector<Chunk> split(const std::vector<char>& buf, int parts) {
  const char* base = buf.data();
  const size_t n = buf.size() - 1;
  std::vector<Chunk> cs;
  size_t at = 0;
  for (int i = 0; i < parts && at < n; ++i) {
    size_t end = i + 1 == parts ? n : std::max(at, n * (size_t)(i + 1) / (size_t)parts);
    while (end < n && base[end - 1] != '\n') ++end;  // extend to the end of the line
    if (end <= at) continue;
    Chunk c;
    c.b = base + at;
    c.e = base + end;
    cs.push_back(c);
    at = end;
  }
  return cs;
}

inline const char* skip_blank(const char* p, const char* e) {
  while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) ++p;
  return p;
}

// Visit every sample line of a chunk: fn(label, pairs...) through a small state machine.
// Returns false with c.err set on a malformed line.
template <class OnRow, class OnPair>
bool walk(Chunk& c, OnRow on_row, OnPair on_pair) {
  const char* p = c.b;
  int64_t line = c.first_line;
  while (p < c.e) {
    const char* eol = static_cast<const char*>(std::memchr(p, '\n', (size_t)(c.e - p)));
    if (!eol) eol = c.e;
    const char* hash = static_cast<const char*>(std::memchr(p, '#', (size_t)(eol - p)));
    const char* end = hash ? hash : eol;
    const char* q = skip_blank(p, end);
    if (q < end) {
      // label
      char* stop = nullptr;
      errno = 0;
      const double label = std::strtod(q, &stop);
      if (stop == q || stop > end) {
        c.err = "line " + std::to_string(line) + ": cannot parse the label";
        return false;
      }
      on_row(label);
      q = skip_blank(stop, end);
      if (end - q >= 4 && std::strncmp(q, "qid:", 4) == 0) {   // query id: skipped
        q += 4;
        while (q < end && *q != ' ' && *q != '\t') ++q;
        q = skip_blank(q, end);
      }
      long long prev = -1;
      while (q < end) {
        char* s2 = nullptr;
        const long long idx = std::strtoll(q, &s2, 10);
        if (s2 == q || s2 >= end || *s2 != ':') {
          c.err = "line " + std::to_string(line) + ": expected index:value";
          return false;
        }
        const char* v = s2 + 1;
        char* s3 = nullptr;
        const double val = std::strtod(v, &s3);
        if (s3 == v || s3 > end) {
          c.err = "line " + std::to_string(line) + ": cannot parse a value";
          return false;
        }
        if (idx < 0) {
          c.err = "line " + std::to_string(line) + ": negative feature index";
          return false;
        }
        if (idx <= prev) {                           // load_svmlight_file's ValueError
          c.err = "line " + std::to_string(line) +
                  ": feature indices in SVMlight/LibSVM data file should be sorted and unique";
          return false;
        }
        prev = idx;
        on_pair((int64_t)idx, val);
        q = skip_blank(s3, end);
      }
    }
    p = eol + 1;
    ++line;
  }
  return true;
}

int nthreads_for(int want, size_t bytes) {
  int hw = (int)std::thread::hardware_concurrency();
  int t = want > 0 ? want : std::min(16, std::max(1, hw));
  const int by_size = (int)std::max<size_t>(1, bytes / (1 << 20));   // >= 1 MB per worker
  return std::max(1, std::min(t, by_size));
}

template <class F>
void run_all(std::vector<Chunk>& cs, F f) {
  std::vector<std::thread> th;
  for (size_t i = 1; i < cs.size(); ++i) th.emplace_back([&, i] { f(cs[i]); });
  if (!cs.empty()) f(cs[0]);
  for (auto& t : th) t.join();
}

// first pass: samples per chunk and index range (line numbers first, for the messages)
bool count(std::vector<Chunk>& cs, std::string& err) {
  int64_t line = 1;
  for (auto& c : cs) {
    c.first_line = line;
    line += std::count(c.b, c.e, '\n');
  }
  run_all(cs, [](Chunk& c) {
    int64_t rows = 0, mn = INT64_MAX, mx = -1;
    walk(c, [&](double) { ++rows; }, [&](int64_t i, double) {
      mn = std::min(mn, i);
      mx = std::max(mx, i);
    });
    c.rows = rows;
    c.min_idx = mn;
    c.max_idx = mx;
  });
  for (auto& c : cs) {
    if (!c.err.empty()) {
      err = c.err;
      return false;
    }
  }
  return true;
}

}  // namespace

extern "C" int fs_libsvm_scan(const char* path, int64_t* n_rows, int64_t* min_index, int64_t* max_index) {
  if (!path || !n_rows || !min_index || !max_index) return fs::fail(FS_EINVAL, "fs_libsvm_scan: null pointer");
  std::vector<char> buf;
  if (!read_file(path, buf)) return fs::fail(FS_EINVAL, std::string("fs_libsvm_scan: cannot read ") + path);
  auto cs = split(buf, nthreads_for(0, buf.size()));
  std::string err;
  if (!count(cs, err)) return fs::fail(FS_EINVAL, "fs_libsvm_scan: " + err);
  int64_t rows = 0, mn = INT64_MAX, mx = -1;
  for (auto& c : cs) {
    rows += c.rows;
    mn = std::min(mn, c.min_idx);
    mx = std::max(mx, c.max_idx);
  }
  *n_rows = rows;
  *min_index = mx < 0 ? -1 : mn;
  *max_index = mx;
  return FS_OK;
}

extern "C" int fs_libsvm_read(const char* path, int64_t n_rows, int64_t n_features, int zero_based, float* X,
                              double* y, int nthreads) {
  if (!path || (n_rows > 0 && (!X || !y)) || n_rows < 0 || n_features < 0)
    return fs::fail(FS_EINVAL, "fs_libsvm_read: bad arguments");
  std::vector<char> buf;
  if (!read_file(path, buf)) return fs::fail(FS_EINVAL, std::string("fs_libsvm_read: cannot read ") + path);
  auto cs = split(buf, nthreads_for(nthreads, buf.size()));
  std::string err;
  if (!count(cs, err)) return fs::fail(FS_EINVAL, "fs_libsvm_read: " + err);
  int64_t rows = 0, mn = INT64_MAX;
  for (auto& c : cs) {
    rows += c.rows;
    mn = std::min(mn, c.min_idx);
  }
  if (rows != n_rows)
    return fs::fail(FS_EINVAL, "fs_libsvm_read: the file has " + std::to_string(rows) + " samples, not " +
                                   std::to_string(n_rows));
  const int64_t off = zero_based == 1 ? 0 : (zero_based == 0 ? 1 : (mn == 0 ? 0 : 1));
  std::vector<int64_t> row0(cs.size(), 0);
  for (size_t i = 1; i < cs.size(); ++i) row0[i] = row0[i - 1] + cs[i - 1].rows;
  std::fill(X, X + n_rows * n_features, 0.0f);
  std::vector<std::string> errs(cs.size());
  std::vector<std::thread> th;
  auto work = [&](size_t i) {
    Chunk& c = cs[i];
    int64_t r = row0[i] - 1;
    std::string bad;
    walk(c, [&](double label) { y[++r] = label; }, [&](int64_t idx, double val) {
      const int64_t col = idx - off;
      if (col < 0 || col >= n_features) {
        if (bad.empty())
          bad = "sample " + std::to_string(r) + ": feature index " + std::to_string(idx) + " outside the " +
                std::to_string(n_features) + " columns";
        return;
      }
      X[r * n_features + col] = (float)val;         // the double, rounded once to float32
    });
    errs[i] = bad;
  };
  for (size_t i = 1; i < cs.size(); ++i) th.emplace_back(work, i);
  if (!cs.empty()) work(0);
  for (auto& t : th) t.join();
  for (auto& e : errs)
    if (!e.empty()) return fs::fail(FS_EINVAL, "fs_libsvm_read: " + e);
  return FS_OK;
}
