// csv.cpp -- parallel reader with the exact token semantics of cpp:154-222.
#include "csv.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <charconv>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace knnhost {

namespace {

// Calls f(token_begin, token_end) for every token of [b, e) following the
// reference's getline-based splitting; returns the number of tokens.
template <class F>
int64_t for_tokens(const char* b, const char* e, F f) {
  int64_t n = 0;
  const char* line = b;
  while (line < e) {
    const char* nl = (const char*)memchr(line, '\n', (size_t)(e - line));
    const char* le = nl ? nl : e;
    const char* tok = line;
    for (;;) {
      const char* comma = (const char*)memchr(tok, ',', (size_t)(le - tok));
      if (comma) {
        f(tok, comma);
        n++;
        tok = comma + 1;
      } else {
        if (le > tok) {  // last segment only if non-empty
          f(tok, le);
          n++;
        }
        break;
      }
    }
    if (!nl) break;
    line = nl + 1;
  }
  return n;
}

// atof / atoi on a token that is not NUL-terminated in the buffer.  The
// common token (a plain decimal that is the whole token) goes through
// std::from_chars, which is correctly rounded like strtod (so the value is
// atof's, bit for bit) and several times faster; anything else -- leading
// blanks or '+', a trailing '\r', hex, inf/nan spellings, trailing garbage --
// falls back to atof itself.
inline double tok_atof_slow(const char* b, const char* e) {
  char buf[128];
  size_t len = (size_t)(e - b);
  if (len < sizeof buf) {
    memcpy(buf, b, len);
    buf[len] = 0;
    return atof(buf);
  }
  std::string s(b, e);
  return atof(s.c_str());
}
inline double tok_atof(const char* b, const char* e) {
  if (b < e && (*b == '-' || (*b >= '0' && *b <= '9') || *b == '.')) {
    double v;
    const std::from_chars_result r = std::from_chars(b, e, v);
    if (r.ec == std::errc() && r.ptr == e) return v;
  }
  return tok_atof_slow(b, e);
}
inline int tok_atoi(const char* b, const char* e) {
  char buf[128];
  size_t len = (size_t)(e - b);
  if (len < sizeof buf) {
    memcpy(buf, b, len);
    buf[len] = 0;
    return atoi(buf);
  }
  std::string s(b, e);
  return atoi(s.c_str());
}

}  // namespace

CsvResult read_csv(const std::string& path, int dim, bool with_label, int64_t rows, double* data,
                   int32_t* labels, int threads) {
  CsvResult r;
  const int fd = open(path.c_str(), O_RDONLY);
  if (fd < 0) {
    r.error = "cannot open " + path;
    return r;
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < 0) {
    close(fd);
    r.error = "cannot size " + path;
    return r;
  }
  const size_t sz = (size_t)st.st_size;
  std::string buf;
  buf.resize(sz);
  if (threads < 1) threads = 1;
  if (sz < (1u << 20)) threads = 1;
  {
    // the read itself in parallel (pread of equal byte ranges)
    std::vector<std::thread> th;
    std::vector<int> bad(threads, 0);
    for (int t = 0; t < threads; t++)
      th.emplace_back([&, t] {
        size_t o = sz * t / threads;
        const size_t end = sz * (t + 1) / threads;
        while (o < end) {
          const ssize_t got = pread(fd, &buf[o], end - o, (off_t)o);
          if (got <= 0) {
            bad[t] = 1;
            return;
          }
          o += (size_t)got;
        }
      });
    for (auto& x : th) x.join();
    close(fd);
    for (int t = 0; t < threads; t++)
      if (bad[t]) {
        r.error = "short read on " + path;
        return r;
      }
  }
  const char* b = buf.data();
  const char* e = b + buf.size();
  // chunk boundaries just after a '\n'
  std::vector<const char*> cut(threads + 1);
  cut[0] = b;
  cut[threads] = e;
  for (int t = 1; t < threads; t++) {
    const char* p = b + (size_t)buf.size() * t / threads;
    if (p < cut[t - 1]) p = cut[t - 1];
    const char* nl = (const char*)memchr(p, '\n', (size_t)(e - p));
    cut[t] = nl ? nl + 1 : e;
  }
  std::vector<int64_t> cnt(threads, 0), first(threads + 1, 0);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++)
      th.emplace_back([&, t] { cnt[t] = for_tokens(cut[t], cut[t + 1], [](const char*, const char*) {}); });
    for (auto& x : th) x.join();
  }
  for (int t = 0; t < threads; t++) first[t + 1] = first[t] + cnt[t];
  const int64_t cap = with_label ? rows * (dim + 1) : rows * dim;
  {
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++)
      th.emplace_back([&, t] {
        int64_t c = first[t];
        for_tokens(cut[t], cut[t + 1], [&](const char* tb, const char* te) {
          if (c < cap) {
            if (with_label) {
              const int64_t row = c / (dim + 1);
              if (c % (dim + 1) == 0) labels[row] = tok_atoi(tb, te);
              else data[c - row - 1] = tok_atof(tb, te);
            } else {
              data[c] = tok_atof(tb, te);
            }
          }
          c++;
        });
      });
    for (auto& x : th) x.join();
  }
  r.tokens = first[threads];
  r.ok = true;
  return r;
}

}  // namespace knnhost
