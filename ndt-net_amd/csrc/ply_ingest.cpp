// ply_ingest.cpp -- native ASCII-PLY reader (include/ndnet_ingest.h), the
// parsing half of CARLA_Seg.get_data_pcl (ndnet/datasets/CARLA_Seg.py:97-136).
// The file is memory-mapped, the data lines are split into newline-aligned
// byte ranges, and each range is parsed by its own thread into the output
// arrays at the range's first line index (a counting pass first).  Numbers go
// through std::from_chars (correctly rounded decimal -> double, like Python's
// float()); the class tag is the line's last token as an integer (int()).
#include <charconv>
#include <cstdint>
#include <cstring>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../../include/ndnet_ingest.h"

namespace {

struct Mapped {
  const char* p = nullptr;
  size_t n = 0;
  int fd = -1;
  bool open(const char* path) {
    fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0) return false;
    n = (size_t)st.st_size;
    if (n == 0) return true;
    void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) return false;
    p = (const char*)m;
    return true;
  }
  ~Mapped() {
    if (p) munmap((void*)p, n);
    if (fd >= 0) close(fd);
  }
};

// Offset just past the header's num_header_lines lines (the reference slices
// readlines()[num_header_lines:]).
size_t skip_header(const Mapped& m, int lines) {
  size_t o = 0;
  for (int i = 0; i < lines && o < m.n; i++) {
    const void* nl = memchr(m.p + o, '\n', m.n - o);
    o = nl ? (size_t)((const char*)nl - m.p) + 1 : m.n;
  }
  return o;
}

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

// A line is a data line unless it is all whitespace (Python's strip().split()
// of a blank line is empty and data[0] would raise; scans end with a newline,
// so the only blank line in practice is the final "").
inline bool blank(const char* a, const char* b) {
  for (; a < b; a++)
    if (!is_space(*a)) return false;
  return true;
}

uint64_t count_lines(const char* a, const char* b) {
  uint64_t c = 0;
  while (a < b) {
    const char* nl = (const char*)memchr(a, '\n', (size_t)(b - a));
    const char* e = nl ? nl : b;
    if (!blank(a, e)) c++;
    a = nl ? nl + 1 : b;
  }
  return c;
}

// Python float() accepts a leading '+', and int() surrounding whitespace and
// a leading '+': from_chars does not take '+', so it is skipped here.
inline const char* parse_double(const char* a, const char* e, double& v) {
  if (a < e && *a == '+') a++;
  auto r = std::from_chars(a, e, v);
  if (r.ec != std::errc() || (r.ptr < e && !is_space(*r.ptr))) return nullptr;
  return r.ptr;
}

// 0 ok, else an NDNET_PLY_ERR_* code; *bad = the failing line index.
int parse_range(const char* a, const char* b, uint64_t line0, int num_classes, double* xyz, uint16_t* cls,
                uint64_t* bad) {
  uint64_t i = line0;
  while (a < b) {
    const char* nl = (const char*)memchr(a, '\n', (size_t)(b - a));
    const char* e = nl ? nl : b;
    if (!blank(a, e)) {
      const char* q = a;
      double v[3];
      int ntok = 0;
      for (int k = 0; k < 3; k++) {
        while (q < e && is_space(*q)) q++;
        q = q < e ? parse_double(q, e, v[k]) : nullptr;
        if (!q) {
          *bad = i;
          return NDNET_PLY_ERR_PARSE;
        }
        ntok++;
      }
      // the last token of the line
      const char* t1 = e;
      while (t1 > q && is_space(t1[-1])) t1--;
      const char* t0 = t1;
      while (t0 > q && !is_space(t0[-1])) t0--;
      if (t0 == t1) {  // fewer than four tokens: data[-1] would be z, int("1.5") raises
        *bad = i;
        return NDNET_PLY_ERR_PARSE;
      }
      if (*t0 == '+') t0++;
      long long tag = 0;
      auto r = std::from_chars(t0, t1, tag);
      if (r.ec != std::errc() || r.ptr != t1) {
        *bad = i;
        return NDNET_PLY_ERR_PARSE;
      }
      if (tag > num_classes || tag < 0) {  // CARLA_Seg.py:126-127; a negative tag fails the uint16 cast (:141)
        *bad = i;
        return NDNET_PLY_ERR_CLASS;
      }
      xyz[3 * i + 0] = v[0];
      xyz[3 * i + 1] = v[1];
      xyz[3 * i + 2] = v[2];
      cls[i] = (uint16_t)tag;
      i++;
    }
    a = nl ? nl + 1 : b;
  }
  return 0;
}

}  // namespace

extern "C" {

int ndnet_ply_count(const char* path, int num_header_lines, uint64_t* n_out) {
  if (!path || !n_out || num_header_lines < 0) return -20;
  Mapped m;
  if (!m.open(path)) return NDNET_PLY_ERR_IO;
  const size_t o = skip_header(m, num_header_lines);
  *n_out = count_lines(m.p + o, m.p + m.n);
  return 0;
}

int ndnet_ply_read(const char* path, int num_header_lines, int num_classes, double* xyz, uint16_t* cls,
                   uint64_t capacity, uint64_t* n_out, int threads) {
  if (!path || !xyz || !cls || !n_out || num_header_lines < 0) return -20;
  Mapped m;
  if (!m.open(path)) return NDNET_PLY_ERR_IO;
  const size_t o = skip_header(m, num_header_lines);
  const char* base = m.p + o;
  const size_t len = m.n - o;
  int T = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
  if (T < 1) T = 1;
  if ((size_t)T > len / 65536 + 1) T = (int)(len / 65536 + 1);  // >= 64 KB per thread
  // newline-aligned ranges
  std::vector<const char*> cut(T + 1);
  cut[0] = base;
  cut[T] = base + len;
  for (int t = 1; t < T; t++) {
    const char* c = base + len * t / T;
    if (c < cut[t - 1]) c = cut[t - 1];
    const void* nl = memchr(c, '\n', (size_t)(base + len - c));
    cut[t] = nl ? (const char*)nl + 1 : base + len;
  }
  std::vector<uint64_t> cnt(T), first(T + 1, 0);
  std::vector<int> rc(T, 0);
  std::vector<uint64_t> bad(T, 0);
  {
    std::vector<std::thread> pool;
    for (int t = 0; t < T; t++) pool.emplace_back([&, t] { cnt[t] = count_lines(cut[t], cut[t + 1]); });
    for (auto& th : pool) th.join();
  }
  for (int t = 0; t < T; t++) first[t + 1] = first[t] + cnt[t];
  if (first[T] > capacity) {
    *n_out = first[T];
    return NDNET_PLY_ERR_CAP;
  }
  {
    std::vector<std::thread> pool;
    for (int t = 0; t < T; t++)
      pool.emplace_back([&, t] { rc[t] = parse_range(cut[t], cut[t + 1], first[t], num_classes, xyz, cls, &bad[t]); });
    for (auto& th : pool) th.join();
  }
  for (int t = 0; t < T; t++)
    if (rc[t]) {  // the first failing line in file order, as the reference's loop raises there
      *n_out = bad[t];
      return rc[t];
    }
  *n_out = first[T];
  return 0;
}

}  // extern "C"
