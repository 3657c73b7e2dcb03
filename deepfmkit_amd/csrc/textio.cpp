// textio.cpp — the reference's raw_data / fit_data text formats on the host side
// of libdfmi.so: header parse, multi-threaded numeric column reader, fit_data
// writer. Host C++ only (no HIP); declared in include/dfmi.h.
//
// Reference (file:line in /root/reference):
//   DeepFitFramework.parse_header ...... core.py:129-174  -> dfmi_txt_parse_header
//   DeepFitFramework.load_raw .......... core.py:259-286  -> dfmi_txt_read (mode DFMI_TXT_SINGLE_SPACE:
//                                                           pandas.read_csv(sep=' ', skiprows=13, usecols=[c]))
//   DeepFitFramework.load_fit .......... core.py:288-332  -> dfmi_txt_read (mode DFMI_TXT_WHITESPACE:
//                                                           numpy.genfromtxt(skip_header=13, invalid_raise=False))
//   DeepFitObject.to_txt ............... data.py:178-208  -> dfmi_fit_txt_write (Python str(float) digits)
//
// Fit files are parsed with std::from_chars (correctly rounded, like CPython's
// float() that genfromtxt uses), raw files with a restatement of pandas' default
// converter (pandas_xstrtod: load_raw reads through pandas.read_csv), and numbers
// are printed with
// std::to_chars in CPython's repr() layout, so a file written here is byte-identical
// to the reference's writer (the header text comes formatted from Python, which
// knows the header fields' Python types) and every value reads back bit-exact.
#include <algorithm>
#include <array>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <system_error>
#include <thread>
#include <vector>

#include <sys/stat.h>

#include "../../include/dfmi.h"

namespace {

thread_local std::string g_txt_err;

int default_threads() {
  const unsigned h = std::thread::hardware_concurrency();
  return h == 0 ? 1 : (h > 16 ? 16 : (int)h);
}

int txt_fail(int code, const std::string& msg) {
  g_txt_err = msg;
  return code;
}

// The whole file in memory (not zero-filled first: the read overwrites it all).
struct Buf {
  std::unique_ptr<char[]> p;
  size_t n = 0;
  const char* data() const { return p.get(); }
  size_t size() const { return n; }
};

struct File {
  Buf buf;
  int load(const char* path) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return txt_fail(DFMI_ERR_ARG, std::string("cannot open ") + path);
    std::fseek(f, 0, SEEK_END);
    const long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    buf.n = n > 0 ? (size_t)n : 0;
    buf.p.reset(new char[buf.n > 0 ? buf.n : 1]);
    const size_t got = n > 0 ? std::fread(buf.p.get(), 1, (size_t)n, f) : 0;
    std::fclose(f);
    if ((long)got != n) return txt_fail(DFMI_ERR_ARG, std::string("short read: ") + path);
    return DFMI_OK;
  }
};

// Fields of one line. SINGLE_SPACE: every ' ' separates (pandas sep=' ': two
// spaces make an empty field). WHITESPACE: runs of blanks separate, leading and
// trailing blanks ignored (numpy.genfromtxt with delimiter=None). '\r' is blank.
template <typename F>
int for_fields(const char* s, const char* e, int mode, F&& f) {
  if (e > s && e[-1] == '\r') --e;
  int k = 0;
  if (mode == DFMI_TXT_SINGLE_SPACE) {
    const char* a = s;
    for (const char* p = s;; ++p) {
      if (p == e || *p == ' ') {
        f(k++, a, p);
        if (p == e) break;
        a = p + 1;
      }
    }
    return k;
  }
  const char* p = s;
  while (true) {
    while (p < e && (*p == ' ' || *p == '\t')) ++p;
    if (p >= e) break;
    const char* a = p;
    while (p < e && *p != ' ' && *p != '\t') ++p;
    f(k++, a, p);
  }
  return k;
}

double parse_double(const char* a, const char* b) {
  while (a < b && *a == '+') ++a;  // from_chars takes no leading '+'
  double v = NAN;
  if (a == b) return NAN;
  const auto r = std::from_chars(a, b, v);
  if (r.ec != std::errc() || r.ptr != b) {
    // "nan", "inf" spellings from_chars missed, anything else is missing data
    std::string t(a, b);
    for (auto& ch : t) ch = (char)std::tolower((unsigned char)ch);
    if (t == "nan" || t == "-nan") return NAN;
    if (t == "inf" || t == "infinity") return INFINITY;
    if (t == "-inf" || t == "-infinity") return -INFINITY;
    return NAN;
  }
  return v;
}

// pandas' default C-engine float converter (read_csv float_precision=None/'high',
// pandas/_libs/src/parser/tokenizer.c precise_xstrtod), restated: up to 17
// significant digits accumulated in a double, the rest of the integer digits
// counted into the exponent, then one multiplication or division by a correctly
// rounded power of ten (two for subnormal results). It is not correctly rounded
// (~1/3 of 17-digit repr() values come out 1 ulp off); load_raw reads raw files
// through it, so the raw reader reproduces it bit for bit — pinned against pandas
// itself by tests/test_textio.py. Returns false if [a, b) is not a number.
const double* pow10_table() {
  // built once, thread-safely (the parse threads call this concurrently)
  static const std::array<double, 309> e = [] {
    std::array<double, 309> t{};
    for (int i = 0; i <= 308; ++i) {
      char buf[16];
      std::snprintf(buf, sizeof buf, "1e%d", i);
      t[(size_t)i] = std::strtod(buf, nullptr);
    }
    return t;
  }();
  return e.data();
}

bool pandas_xstrtod(const char* p, const char* end, double* out) {
  const double* e = pow10_table();
  double number = 0.0;
  int exponent = 0, num_digits = 0, num_decimals = 0;
  const int max_digits = 17;
  bool negative = false;
  while (p < end && (*p == ' ' || *p == '\t')) ++p;  // leading blanks
  if (p < end && (*p == '-' || *p == '+')) {
    negative = *p == '-';
    ++p;
  }
  const char* digits0 = p;
  while (p < end && *p >= '0' && *p <= '9') {
    if (num_digits < max_digits) {
      number = number * 10. + (*p - '0');
      ++num_digits;
    } else {
      ++exponent;
    }
    ++p;
  }
  if (p < end && *p == '.') {
    ++p;
    while (num_digits < max_digits && p < end && *p >= '0' && *p <= '9') {
      number = number * 10. + (*p - '0');
      ++p;
      ++num_digits;
      ++num_decimals;
    }
    if (num_digits >= max_digits)
      while (p < end && *p >= '0' && *p <= '9') ++p;
    exponent -= num_decimals;
  }
  if (p == digits0 || (p == digits0 + 1 && *digits0 == '.')) return false;  // no digits
  if (negative) number = -number;
  if (p < end && (*p == 'e' || *p == 'E')) {
    const char* q = p + 1;
    bool eneg = false;
    if (q < end && (*q == '-' || *q == '+')) {
      eneg = *q == '-';
      ++q;
    }
    if (q < end && *q >= '0' && *q <= '9') {
      int n = 0;
      while (q < end && *q >= '0' && *q <= '9') {
        if (n < 100000) n = n * 10 + (*q - '0');
        ++q;
      }
      exponent += eneg ? -n : n;
      p = q;
    }
  }
  if (exponent > 308) {
    number = number == 0.0 ? number : (number < 0 ? -HUGE_VAL : HUGE_VAL);
  } else if (exponent > 0) {
    number *= e[exponent];
  } else if (exponent < -308) {  // subnormal
    if (exponent < -616) {
      number = 0.;
    } else {
      number /= e[-308 - exponent];
      number /= e[308];
    }
  } else {
    number /= e[-exponent];
  }
  while (p < end && (*p == ' ' || *p == '\t')) ++p;  // trailing blanks
  if (p != end) return false;
  *out = number;
  return true;
}

double parse_pandas(const char* a, const char* b) {
  double v;
  if (a == b) return NAN;
  if (pandas_xstrtod(a, b, &v)) return v;
  std::string t(a, b);  // pandas' NA / inf spellings
  for (auto& ch : t) ch = (char)std::tolower((unsigned char)ch);
  if (t == "inf" || t == "+inf" || t == "infinity" || t == "+infinity") return INFINITY;
  if (t == "-inf" || t == "-infinity") return -INFINITY;
  return NAN;
}

bool is_comment(const char* s, const char* e, int mode) {
  if (mode != DFMI_TXT_WHITESPACE) return false;  // genfromtxt: comments='#'
  while (s < e && (*s == ' ' || *s == '\t')) ++s;
  return s < e && *s == '#';
}

bool is_blank(const char* s, const char* e) {
  for (; s < e; ++s)
    if (*s != ' ' && *s != '\t' && *s != '\r' && *s != '\n') return false;
  return true;
}

// Every line after `skip`, indexed and classified in parallel over byte ranges cut
// at line ends: st = line start offsets, nf = fields of a data line, -1 for a
// blank or comment line (the caller applies the row rules that need the order,
// e.g. genfromtxt's "same field count as the first row").
struct Scan {
  std::vector<size_t> st;
  std::vector<int> nf;
};

// File identity for the shape -> read hand-over: size + modification time.
struct Stamp {
  long long size = -1, sec = 0, nsec = 0;
  bool operator==(const Stamp& o) const { return size == o.size && sec == o.sec && nsec == o.nsec; }
};

bool stamp_of(const char* path, Stamp* s) {
  struct stat st;
  if (stat(path, &st) != 0) return false;
  s->size = (long long)st.st_size;
  s->sec = (long long)st.st_mtim.tv_sec;
  s->nsec = (long long)st.st_mtim.tv_nsec;
  return true;
}

void scan_lines(const Buf& b, int skip, int mode, int threads, Scan* sc) {
  const size_t n = b.size();
  size_t i0 = 0;
  for (int k = 0; k < skip && i0 < n; ++k) {
    const void* p = std::memchr(b.data() + i0, '\n', n - i0);
    i0 = p ? (size_t)((const char*)p - b.data()) + 1 : n;
  }
  const int nt = (threads > 1 && n - i0 > ((size_t)1 << 20)) ? threads : 1;
  // range t starts at the first line start at or after i0 + t*(n-i0)/nt
  std::vector<size_t> cut((size_t)nt + 1, n);
  cut[0] = i0;
  for (int t = 1; t < nt; ++t) {
    size_t c = i0 + (n - i0) / (size_t)nt * (size_t)t;
    const void* p = std::memchr(b.data() + c - 1, '\n', n - (c - 1));
    cut[(size_t)t] = p ? (size_t)((const char*)p - b.data()) + 1 : n;
  }
  for (int t = 1; t <= nt; ++t) cut[(size_t)t] = std::max(cut[(size_t)t], cut[(size_t)t - 1]);
  std::vector<std::vector<size_t>> lst((size_t)nt);
  std::vector<std::vector<int>> lnf((size_t)nt);
  auto work = [&](int t) {
    size_t i = cut[(size_t)t];
    const size_t hi = cut[(size_t)t + 1];
    auto& S = lst[(size_t)t];
    auto& F = lnf[(size_t)t];
    while (i < hi) {
      const void* p = std::memchr(b.data() + i, '\n', n - i);
      const size_t nx = p ? (size_t)((const char*)p - b.data()) + 1 : n;
      const char* s0 = b.data() + i;
      const char* e = b.data() + nx;
      if (e > s0 && e[-1] == '\n') --e;
      S.push_back(i);
      F.push_back((is_blank(s0, e) || is_comment(s0, e, mode))
                      ? -1
                      : for_fields(s0, e, mode, [](int, const char*, const char*) {}));
      i = nx;
    }
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t) pool.emplace_back(work, t);
    for (auto& th : pool) th.join();
  }
  size_t tot = 0;
  for (auto& v : lst) tot += v.size();
  sc->st.reserve(tot);
  sc->nf.reserve(tot);
  for (int t = 0; t < nt; ++t) {
    sc->st.insert(sc->st.end(), lst[(size_t)t].begin(), lst[(size_t)t].end());
    sc->nf.insert(sc->nf.end(), lnf[(size_t)t].begin(), lnf[(size_t)t].end());
  }
}

// CPython repr(float): shortest round-trip digits; fixed notation when the
// decimal exponent is in [-4, 16), with ".0" for integral values; otherwise
// d[.ddd]e±XX with at least two exponent digits.
void py_repr(double v, std::string* out) {
  if (std::isnan(v)) {
    *out += "nan";
    return;
  }
  if (std::isinf(v)) {
    *out += v < 0 ? "-inf" : "inf";
    return;
  }
  char sci[64];
  auto r = std::to_chars(sci, sci + sizeof sci, v, std::chars_format::scientific);
  *r.ptr = 0;
  // sci = [-]d[.ddd]e(+|-)XX
  std::string s(sci);
  bool neg = false;
  if (s[0] == '-') {
    neg = true;
    s.erase(0, 1);
  }
  const size_t epos = s.find('e');
  std::string mant = s.substr(0, epos);
  const int exp10 = std::atoi(s.c_str() + epos + 1);
  std::string digits;
  for (char ch : mant)
    if (ch != '.') digits += ch;
  if (neg) *out += '-';
  if (exp10 >= -4 && exp10 < 16) {
    const int nd = (int)digits.size();
    if (exp10 >= 0) {
      if (nd <= exp10 + 1) {
        *out += digits;
        out->append((size_t)(exp10 + 1 - nd), '0');
        *out += ".0";
      } else {
        *out += digits.substr(0, (size_t)exp10 + 1);
        *out += '.';
        *out += digits.substr((size_t)exp10 + 1);
      }
    } else {
      *out += "0.";
      out->append((size_t)(-exp10 - 1), '0');
      *out += digits;
    }
    return;
  }
  *out += digits.substr(0, 1);
  if (digits.size() > 1) {
    *out += '.';
    *out += digits.substr(1);
  }
  char eb[16];
  std::snprintf(eb, sizeof eb, "e%c%02d", exp10 < 0 ? '-' : '+', exp10 < 0 ? -exp10 : exp10);
  *out += eb;
}

// core.py:149-150: for lines 2..10 keep only the characters of '1234567890.'.
std::string digits_only(const std::string& line) {
  std::string o;
  for (char ch : line)
    if ((ch >= '0' && ch <= '9') || ch == '.') o += ch;
  return o;
}

// What dfmi_txt_shape loaded, for the dfmi_txt_read of the same file that follows
// on this thread (textio.read_columns calls them in that order); dropped by the read.
struct Loaded {
  File f;
  Scan sc;
  std::string path;
  int skip = -1, mode = -1;
  Stamp stamp;
};
thread_local Loaded g_loaded;

}  // namespace

extern "C" {

const char* dfmi_txt_last_error(void) { return g_txt_err.c_str(); }

int dfmi_txt_parse_header(const char* path, int32_t kind, dfmi_txt_header* hdr) {
  g_txt_err.clear();
  if (!path || !hdr || (kind != DFMI_TXT_RAW && kind != DFMI_TXT_FIT)) return txt_fail(DFMI_ERR_ARG, "bad argument");
  FILE* f = std::fopen(path, "rb");
  if (!f) return txt_fail(DFMI_ERR_ARG, std::string("cannot open ") + path);
  std::vector<std::string> lines;
  char buf[4096];
  for (int i = 0; i < 11; ++i) {
    std::string l;
    if (std::fgets(buf, sizeof buf, f)) l = buf;
    lines.push_back(l);
  }
  std::fclose(f);
  std::vector<std::string> v;
  for (int i = 2; i < 11; ++i) v.push_back(digits_only(lines[i]));
  memset(hdr, 0, sizeof(*hdr));
  hdr->kind = kind;
  // int(...) / float(...) of the filtered strings, as core.py:152-163 does; an
  // empty or malformed field is an error there (ValueError) and here
  auto to_i64 = [&](const std::string& t, int64_t* o) {
    if (t.empty() || t.find('.') != std::string::npos) return false;
    const auto r = std::from_chars(t.data(), t.data() + t.size(), *o);
    return r.ec == std::errc() && r.ptr == t.data() + t.size();
  };
  auto to_f = [&](const std::string& t, double* o) {
    if (t.empty()) return false;
    const auto r = std::from_chars(t.data(), t.data() + t.size(), *o);
    return r.ec == std::errc() && r.ptr == t.data() + t.size();
  };
  int64_t ch = 0, n = 0, R = 0;
  if (!to_i64(v[0], &ch) || !to_i64(v[1], &hdr->t0) || !to_f(v[2], &hdr->f_samp) || !to_f(v[3], &hdr->f_mod))
    return txt_fail(DFMI_ERR_ARG, std::string("malformed header (lines 3-6): ") + path);
  hdr->channels = (int32_t)ch;
  if (kind == DFMI_TXT_FIT) {
    if (!to_i64(v[4], &n) || !to_i64(v[5], &R) || !to_f(v[6], &hdr->fs))
      return txt_fail(DFMI_ERR_ARG, std::string("malformed fit header (lines 7-9): ") + path);
    hdr->n = (int32_t)n;
    hdr->R = (int32_t)R;
  }
  return DFMI_OK;
}

int dfmi_txt_shape(const char* path, int32_t skip, int32_t mode, int64_t* rows, int32_t* cols) {
  g_txt_err.clear();
  if (!path || !rows || !cols || skip < 0) return txt_fail(DFMI_ERR_ARG, "bad argument");
  Loaded& L = g_loaded;
  L = Loaded();
  int rc = L.f.load(path);
  if (rc) return rc;
  scan_lines(L.f.buf, skip, mode, default_threads(), &L.sc);
  if (stamp_of(path, &L.stamp)) {  // kept for the dfmi_txt_read that follows
    L.path = path;
    L.skip = skip;
    L.mode = mode;
  }
  const File& f = L.f;
  const Scan& sc = L.sc;
  (void)f;
  int64_t nr = 0;
  int32_t nc = 0, first = -1;
  for (size_t i = 0; i < sc.st.size(); ++i) {
    const int k = sc.nf[i];
    if (k < 0) continue;
    if (mode == DFMI_TXT_WHITESPACE) {
      if (first < 0) first = k;
      if (k != first) continue;  // genfromtxt(invalid_raise=False) drops such rows
    }
    if (k > nc) nc = k;
    ++nr;
  }
  *rows = nr;
  *cols = nc;
  return DFMI_OK;
}

int dfmi_txt_read(const char* path, int32_t skip, int32_t mode, int32_t ncol, const int32_t* cols, double* out,
                  int64_t rows, int32_t threads) {
  g_txt_err.clear();
  if (!path || skip < 0 || ncol < 0 || (ncol && (!cols || !out)) || rows < 0) return txt_fail(DFMI_ERR_ARG, "bad argument");
  // the file and its line scan as dfmi_txt_shape left them (same path, size and
  // modification time, same skip / mode), else loaded and scanned here
  File f;
  Scan sc;
  Stamp now;
  Loaded& L = g_loaded;
  if (!L.path.empty() && L.path == path && L.skip == skip && L.mode == mode && stamp_of(path, &now) &&
      now == L.stamp) {
    f = std::move(L.f);
    sc = std::move(L.sc);
  } else {
    int rc = f.load(path);
    if (rc) return rc;
    // pass 1: line index and classification (parallel)
    scan_lines(f.buf, skip, mode, threads, &sc);
  }
  L = Loaded();
  // then the row numbers in file order (serial over the per-line field counts)
  const std::vector<size_t>& st = sc.st;
  std::vector<int64_t> row_of(st.size(), -1);
  int64_t nr = 0;
  int first = -1;
  auto line_end = [&](size_t i) {
    const char* e = f.buf.data() + (i + 1 < st.size() ? st[i + 1] : f.buf.size());
    if (e > f.buf.data() + st[i] && e[-1] == '\n') --e;
    return e;
  };
  for (size_t i = 0; i < st.size(); ++i) {
    const int k = sc.nf[i];
    if (k < 0) continue;
    if (mode == DFMI_TXT_WHITESPACE) {
      if (first < 0) first = k;
      if (k != first) continue;
    }
    if (nr < rows) row_of[i] = nr;
    ++nr;
  }
  if (nr != rows) return txt_fail(DFMI_ERR_ARG, "row count changed or does not match dfmi_txt_shape");
  std::vector<int> slot(1, -1);
  int maxc = -1;
  for (int k = 0; k < ncol; ++k) maxc = cols[k] > maxc ? cols[k] : maxc;
  slot.assign((size_t)(maxc + 1), -1);
  for (int k = 0; k < ncol; ++k)
    if (cols[k] >= 0) slot[(size_t)cols[k]] = k;
  for (int64_t k = 0; k < (int64_t)ncol * rows; ++k) out[k] = NAN;
  // pass 2 (parallel): parse the requested columns of every data row
  const int nt = threads > 0 ? threads : 1;
  auto work = [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      const int64_t r = row_of[i];
      if (r < 0) continue;
      for_fields(f.buf.data() + st[i], line_end(i), mode, [&](int c, const char* a, const char* b) {
        if (c <= maxc && slot[(size_t)c] >= 0)
          out[(int64_t)slot[(size_t)c] * rows + r] = mode == DFMI_TXT_SINGLE_SPACE ? parse_pandas(a, b) : parse_double(a, b);
      });
    }
  };
  if (nt == 1 || st.size() < 4096) {
    work(0, st.size());
  } else {
    std::vector<std::thread> pool;
    const size_t chunk = (st.size() + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
      const size_t lo = (size_t)t * chunk, hi = lo + chunk < st.size() ? lo + chunk : st.size();
      if (lo < hi) pool.emplace_back(work, lo, hi);
    }
    for (auto& th : pool) th.join();
  }
  return DFMI_OK;
}

int dfmi_fit_txt_write(const char* path, const char* header, const double* ssq, const double* amp, const double* m,
                       const double* phi, const double* psi, const double* dc, int64_t n) {
  g_txt_err.clear();
  if (!path || !header || n < 0 || (n && (!ssq || !amp || !m || !phi || !psi || !dc)))
    return txt_fail(DFMI_ERR_ARG, "bad argument");
  // data.py:198-207: str(v) + ' ' per column, then '\n'; row ranges formatted in
  // parallel into their own strings, written in order
  const int nt = n >= 4096 ? default_threads() : 1;
  std::vector<std::string> part((size_t)nt);
  auto fmt = [&](int t) {
    const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
    std::string& o = part[(size_t)t];
    o.reserve((size_t)(hi - lo) * 120);
    for (int64_t i = lo; i < hi; ++i) {
      const double v[6] = {ssq[i], amp[i], m[i], phi[i], psi[i], dc[i]};
      for (int c = 0; c < 6; ++c) {
        py_repr(v[c], &o);
        o += ' ';
      }
      o += '\n';
    }
  };
  if (nt == 1) {
    fmt(0);
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < nt; ++t) pool.emplace_back(fmt, t);
    for (auto& th : pool) th.join();
  }
  FILE* f = std::fopen(path, "wb");
  if (!f) return txt_fail(DFMI_ERR_ARG, std::string("cannot write ") + path);
  const size_t hl = std::strlen(header);
  bool ok = std::fwrite(header, 1, hl, f) == hl;
  for (const auto& o : part) ok = ok && std::fwrite(o.data(), 1, o.size(), f) == o.size();
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) return txt_fail(DFMI_ERR_ARG, std::string("short write: ") + path);
  return DFMI_OK;
}

int dfmi_py_repr(double v, char* buf, int32_t cap) {
  std::string s;
  py_repr(v, &s);
  if (!buf || cap <= (int32_t)s.size()) return DFMI_ERR_ARG;
  std::memcpy(buf, s.c_str(), s.size() + 1);
  return (int)s.size();
}

}  // extern "C"
