// Long-format CSV -> dense [F][D][A] panel loader (host C++, libfmx_io.so).
//
// The step in front of the factor-panel path: pipeline.ipynb:71-82 reads
// 2.symbol_features_long.csv / 8.factors_df.csv with pd.read_csv, converts the date column
// with pd.to_datetime and sets a (date, symbol) MultiIndex; the engine then wants the
// panel dense in HBM ([F][D][A] fp64, factormodeling_amd/panel.py).  pandas does this in
// one thread and builds Python objects per row; here the file is mmapped, cut into
// newline-aligned chunks parsed by N threads, and the values scattered straight into the
// dense layout (or a row-major copy for the drop-in DataFrame).
//
// Float fields follow pandas' default parser bit-for-bit (pandas 2.3.3,
// pandas/_libs/src/parser/tokenizer.c precise_xstrtod, called from parsers.pyx
// _try_double_nogil with skip_trailing=1): up to 17 significant digits are accumulated in
// a double (number = number * 10 + digit), the decimal exponent is applied with ONE
// multiply or divide by a correctly rounded power of ten (two divides below 1e-308).  This
// is not correctly rounded (about a quarter of 17-digit repr() strings land 1 ulp away
// from strtod), which is why strtod/from_chars would break parity with the reference.
#include "../../include/fmx_io.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int code, std::string msg) {
  g_err = std::move(msg);
  return code;
}

// 1e0 .. 1e308 exactly as the C compiler rounds the literals in tokenizer.c's table
// (strtod is correctly rounded, as are decimal floating literals).
struct Pow10 {
  double e[309];
  Pow10() {
    char buf[16];
    for (int k = 0; k <= 308; ++k) {
      snprintf(buf, sizeof buf, "1e%d", k);
      e[k] = strtod(buf, nullptr);
    }
  }
};
const Pow10& pow10() {
  static const Pow10 t;
  return t;
}

inline bool is_digit(char c) { return c >= '0' && c <= '9'; }
inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }

// tokenizer.c precise_xstrtod (decimal '.', sci 'E', no thousands separator,
// skip_trailing = 1).  Returns the end pointer; *err set like its ERANGE.
const char* precise_xstrtod(const char* p, const char* end, double* out, int* err) {
  const int max_digits = 17;
  const double* e = pow10().e;
  *err = 0;
  while (p < end && is_space(*p)) ++p;
  bool neg = false;
  if (p < end && (*p == '-' || *p == '+')) {
    neg = *p == '-';
    ++p;
  }
  double number = 0.;
  int exponent = 0, num_digits = 0, num_decimals = 0;
  while (p < end && is_digit(*p)) {
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
    while (num_digits < max_digits && p < end && is_digit(*p)) {
      number = number * 10. + (*p - '0');
      ++p;
      ++num_digits;
      ++num_decimals;
    }
    if (num_digits >= max_digits)
      while (p < end && is_digit(*p)) ++p;
    exponent -= num_decimals;
  }
  if (num_digits == 0) {
    *err = 1;
    *out = 0.0;
    return p;
  }
  if (neg) number = -number;
  if (p < end && (*p == 'e' || *p == 'E')) {
    ++p;
    bool eneg = false;
    if (p < end && (*p == '-' || *p == '+')) {
      eneg = *p == '-';
      ++p;
    }
    int nd = 0, n = 0;
    while (nd < max_digits && p < end && is_digit(*p)) {
      n = n * 10 + (*p - '0');
      ++nd;
      ++p;
    }
    exponent += eneg ? -n : n;
    if (nd == 0) --p;  // tokenizer.c un-consumes the 'e' only (a dangling sign stays eaten)
  }
  if (exponent > 308) {
    *err = 1;
    *out = HUGE_VAL;
    return p;
  } else if (exponent > 0) {
    number *= e[exponent];
  } else if (exponent < -308) {
    if (exponent < -616) {
      number = 0.;
    } else {
      number /= e[-308 - exponent];
      number /= e[308];
    }
  } else {
    number /= e[-exponent];
  }
  if (number == HUGE_VAL || number == -HUGE_VAL) *err = 1;
  while (p < end && is_space(*p)) ++p;
  *out = number;
  return p;
}

// pandas' default na_values (pandas/_libs/parsers.pyx STR_NA_VALUES).
bool is_na(std::string_view f) {
  static const std::unordered_set<std::string_view> na = {
      "", "#N/A", "#N/A N/A", "#NA", "-1.#IND", "-1.#QNAN", "-NaN", "-nan", "1.#IND",
      "1.#QNAN", "<NA>", "N/A", "NA", "NULL", "NaN", "None", "n/a", "nan", "null"};
  return na.count(f) != 0;
}

bool ieq(std::string_view a, const char* b) {
  size_t n = strlen(b);
  if (a.size() != n) return false;
  for (size_t i = 0; i < n; ++i) {
    char c = a[i];
    if (c >= 'A' && c <= 'Z') c = char(c - 'A' + 'a');
    if (c != b[i]) return false;
  }
  return true;
}

// parsers.pyx _try_double_nogil: precise_xstrtod, then the inf spellings.
bool parse_value(std::string_view f, double* v) {
  int err;
  const char* b = f.data();
  const char* end = precise_xstrtod(b, b + f.size(), v, &err);
  if (err == 0 && end != b && end == b + f.size()) return true;
  if (ieq(f, "inf") || ieq(f, "+inf") || ieq(f, "infinity") || ieq(f, "+infinity")) {
    *v = HUGE_VAL;
    return true;
  }
  if (ieq(f, "-inf") || ieq(f, "-infinity")) {
    *v = -HUGE_VAL;
    return true;
  }
  return false;
}

// An int64 literal as pandas' str_to_int64 accepts it (blanks, sign, <= 18 digits here).
bool int_like(std::string_view f) {
  size_t i = 0, n = f.size();
  while (i < n && is_space(f[i])) ++i;
  if (i < n && (f[i] == '-' || f[i] == '+')) ++i;
  size_t d0 = i;
  while (i < n && is_digit(f[i])) ++i;
  size_t nd = i - d0;
  while (i < n && is_space(f[i])) ++i;
  return i == n && nd >= 1 && nd <= 18;
}

int64_t days_from_civil(int64_t y, unsigned m, unsigned d) {
  y -= m <= 2;
  const int64_t era = (y >= 0 ? y : y - 399) / 400;
  const unsigned yoe = unsigned(y - era * 400);
  const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
  const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + int64_t(doe) - 719468;
}

bool digits(std::string_view s, size_t at, size_t n, int64_t* v) {
  if (at + n > s.size()) return false;
  int64_t x = 0;
  for (size_t i = at; i < at + n; ++i) {
    if (!is_digit(s[i])) return false;
    x = x * 10 + (s[i] - '0');
  }
  *v = x;
  return true;
}

// ISO 'YYYY-MM-DD' [('T'|' ') 'HH:MM' [':SS' ['.' fraction]]] -> ns since epoch.
bool parse_date(std::string_view s, int64_t* ns) {
  int64_t y, mo, d, hh = 0, mi = 0, ss = 0, frac = 0;
  if (s.size() < 10 || !digits(s, 0, 4, &y) || s[4] != '-' || !digits(s, 5, 2, &mo) || s[7] != '-' ||
      !digits(s, 8, 2, &d))
    return false;
  if (mo < 1 || mo > 12 || d < 1 || d > 31) return false;
  size_t i = 10;
  if (i < s.size()) {
    if ((s[i] != ' ' && s[i] != 'T') || !digits(s, i + 1, 2, &hh) || i + 3 >= s.size() || s[i + 3] != ':' ||
        !digits(s, i + 4, 2, &mi))
      return false;
    i += 6;
    if (i < s.size()) {
      if (s[i] != ':' || !digits(s, i + 1, 2, &ss)) return false;
      i += 3;
      if (i < s.size()) {
        if (s[i] != '.') return false;
        ++i;
        int64_t scale = 100000000;
        size_t k = 0;
        for (; i < s.size() && is_digit(s[i]); ++i, ++k) {
          if (k < 9) frac += (s[i] - '0') * scale;
          scale /= 10;
        }
        if (k == 0 || i != s.size()) return false;
      }
    }
    if (hh > 23 || mi > 59 || ss > 59) return false;
  }
  const int64_t days = days_from_civil(y, unsigned(mo), unsigned(d));
  *ns = ((days * 24 + hh) * 60 + mi) * 60 * 1000000000LL + ss * 1000000000LL + frac;
  return true;
}

struct Chunk {
  const char* b = nullptr;
  const char* e = nullptr;
  int64_t rows = 0;
  std::vector<int64_t> date_ns;
  std::vector<std::string_view> sym;
  std::vector<double> vals;
  std::vector<uint8_t> not_int;
  std::string err;
};

int pick_threads(int n) {
  if (n > 0) return std::min(n, 64);
  unsigned h = std::thread::hardware_concurrency();
  return int(std::max(1u, std::min(h ? h : 1u, 16u)));
}

template <class Fn>
void parallel_for(int nt, int64_t n, Fn fn) {
  nt = int(std::max<int64_t>(1, std::min<int64_t>(nt, n)));
  if (nt == 1) {
    fn(0, int64_t(0), n);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) {
    int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
    th.emplace_back([=] { fn(t, lo, hi); });
  }
  for (auto& x : th) x.join();
}

}  // namespace

struct fmx_csv {
  void* map = nullptr;
  size_t map_len = 0;
  std::vector<std::string> names;
  std::vector<Chunk> chunks;
  std::vector<int64_t> chunk_row0;
  int64_t n_rows = 0, F = 0, D = 0, A = 0;
  std::vector<int64_t> dates;
  std::vector<std::string_view> symbols;
  std::vector<int64_t> flat;
  std::vector<int32_t> int_cols;
  int32_t per_symbol_sorted = 1;
  int64_t dup_row = -1;
  ~fmx_csv() {
    if (map && map != MAP_FAILED) munmap(map, map_len);
  }
};

namespace {

void parse_chunk(Chunk& c, int ncol, int dcol, int scol, int F) {
  c.not_int.assign(F, 0);
  const char* p = c.b;
  std::vector<std::string_view> f(ncol);
  while (p < c.e) {
    const char* nl = static_cast<const char*>(memchr(p, '\n', size_t(c.e - p)));
    const char* le = nl ? nl : c.e;
    const char* next = nl ? nl + 1 : c.e;
    if (le > p && le[-1] == '\r') --le;
    if (le == p) {  // pandas skip_blank_lines
      p = next;
      continue;
    }
    int k = 0;
    const char* q = p;
    while (true) {
      const char* comma = static_cast<const char*>(memchr(q, ',', size_t(le - q)));
      const char* fe = comma ? comma : le;
      if (k >= ncol) {
        c.err = "data row " + std::to_string(c.rows) + ": more fields than header columns";
        return;
      }
      f[k++] = std::string_view(q, size_t(fe - q));
      if (!comma) break;
      q = comma + 1;
    }
    if (k != ncol) {
      c.err = "data row " + std::to_string(c.rows) + ": " + std::to_string(k) + " fields, header has " +
              std::to_string(ncol);
      return;
    }
    for (int j = 0; j < ncol; ++j)
      if (memchr(f[j].data(), '"', f[j].size())) {
        c.err = "data row " + std::to_string(c.rows) + ": quoted fields are not supported";
        return;
      }
    int64_t ns;
    if (!parse_date(f[dcol], &ns)) {
      c.err = "data row " + std::to_string(c.rows) + ": date '" + std::string(f[dcol]) + "' is not ISO YYYY-MM-DD[ HH:MM[:SS[.f]]]";
      return;
    }
    if (scol >= 0 && is_na(f[scol])) {   // pandas would read a NaN symbol ('NA' is a ticker)
      c.err = "data row " + std::to_string(c.rows) + ": symbol '" + std::string(f[scol]) +
              "' is one of pandas' NA spellings (pandas reads it as NaN): not supported";
      return;
    }
    c.date_ns.push_back(ns);
    c.sym.push_back(scol >= 0 ? f[scol] : std::string_view());
    int v = 0;
    for (int j = 0; j < ncol; ++j) {
      if (j == dcol || j == scol) continue;
      double x;
      if (is_na(f[j])) {
        x = NAN;
        c.not_int[v] = 1;
      } else if (parse_value(f[j], &x)) {
        if (!c.not_int[v] && !int_like(f[j])) c.not_int[v] = 1;
      } else {
        c.err = "data row " + std::to_string(c.rows) + ": value '" + std::string(f[j]) + "' is not numeric";
        return;
      }
      c.vals.push_back(x);
      ++v;
    }
    ++c.rows;
    p = next;
  }
}

// Python repr(float) (float_repr_style 'short', Py_DTSF_ADD_DOT_0): shortest round-trip
// digits; fixed notation when -4 < decpt <= 16, else d[.ddd]e+XX.  pandas' to_csv writes
// float64 cells this way (na_rep '' for NaN).
int py_repr(double x, char* out) {
  if (std::isnan(x)) return 0;
  if (std::isinf(x)) {
    const char* s = x > 0 ? "inf" : "-inf";
    size_t n = strlen(s);
    memcpy(out, s, n);
    return int(n);
  }
  char sci[64];
  auto r = std::to_chars(sci, sci + sizeof sci - 1, x, std::chars_format::scientific);
  *r.ptr = 0;  // to_chars does not terminate; the exponent is read with atoi below
  char* p = sci;
  char* end = r.ptr;
  char* o = out;
  if (*p == '-') {
    *o++ = '-';
    ++p;
  }
  char dg[32];
  int nd = 0;
  for (; p < end && *p != 'e'; ++p)
    if (*p != '.') dg[nd++] = *p;
  int e10 = std::atoi(p + 1);  // x = d1.d2... * 10^e10
  if (nd == 1 && dg[0] == '0') e10 = 0;
  const int decpt = e10 + 1;
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      *o++ = '0';
      *o++ = '.';
      for (int i = 0; i < -decpt; ++i) *o++ = '0';
      for (int i = 0; i < nd; ++i) *o++ = dg[i];
    } else {
      for (int i = 0; i < decpt; ++i) *o++ = i < nd ? dg[i] : '0';
      *o++ = '.';
      if (nd > decpt)
        for (int i = decpt; i < nd; ++i) *o++ = dg[i];
      else
        *o++ = '0';
    }
  } else {
    *o++ = dg[0];
    if (nd > 1) {
      *o++ = '.';
      for (int i = 1; i < nd; ++i) *o++ = dg[i];
    }
    *o++ = 'e';
    *o++ = e10 < 0 ? '-' : '+';
    int ae = e10 < 0 ? -e10 : e10;
    if (ae < 10) *o++ = '0';
    char eb[8];
    auto er = std::to_chars(eb, eb + 8, ae);
    for (char* q = eb; q < er.ptr; ++q) *o++ = *q;
  }
  return int(o - out);
}

std::vector<std::string_view> split_lines(const char* s, int64_t n) {
  std::vector<std::string_view> v;
  if (!s) return v;
  const char* p = s;
  for (int64_t k = 0; k < n; ++k) {
    const char* nl = strchr(p, '\n');
    if (!nl) break;
    v.emplace_back(p, size_t(nl - p));
    p = nl + 1;
  }
  return v;
}

}  // namespace

extern "C" {

int fmx_format_double(double x, char* buf, int32_t cap) {
  char tmp[64];
  int n = py_repr(x, tmp);
  if (!buf || cap < n + 1) return -1;
  memcpy(buf, tmp, size_t(n));
  buf[n] = 0;
  return n;
}

int fmx_csv_write(const char* path, const char* header, const char* date_strs, const char* symbol_strs,
                  const double* X, int64_t F, int64_t D, int64_t A, const uint8_t* present, int nthreads) {
  if (!path || !header || !date_strs || (!X && F * D * A != 0) || F < 0 || D < 0 || A < 0)
    return fail(FMX_IO_ERR_ARG, "bad argument");
  const auto dates = split_lines(date_strs, D);
  const auto syms = split_lines(symbol_strs, A);
  if (int64_t(dates.size()) != D || (symbol_strs && int64_t(syms.size()) != A) || (!symbol_strs && A != 1))
    return fail(FMX_IO_ERR_ARG, "date/symbol string counts do not match D/A");
  FILE* fp = fopen(path, "wb");
  if (!fp) return fail(FMX_IO_ERR_OPEN, std::string("cannot write ") + path + ": " + strerror(errno));
  fputs(header, fp);
  fputc('\n', fp);
  const int nt = pick_threads(nthreads);
  const int64_t DA = D * A;
  const int64_t batch = std::max<int64_t>(nt, 64);  // dates formatted per round
  std::vector<std::string> out(static_cast<size_t>(batch));
  for (int64_t d0 = 0; d0 < D; d0 += batch) {
    const int64_t d1 = std::min(D, d0 + batch);
    parallel_for(nt, d1 - d0, [&](int, int64_t lo, int64_t hi) {
      char num[64];
      for (int64_t i = lo; i < hi; ++i) {
        const int64_t d = d0 + i;
        std::string& s = out[size_t(i)];
        s.clear();
        for (int64_t a = 0; a < A; ++a) {
          const int64_t cell = d * A + a;
          if (present && !present[cell]) continue;
          s.append(dates[size_t(d)]);
          if (symbol_strs) (s += ',').append(syms[size_t(a)]);
          for (int64_t f = 0; f < F; ++f) {
            s += ',';
            s.append(num, size_t(py_repr(X[f * DA + cell], num)));
          }
          s += '\n';
        }
      }
    });
    for (int64_t i = 0; i < d1 - d0; ++i) fwrite(out[size_t(i)].data(), 1, out[size_t(i)].size(), fp);
  }
  if (fclose(fp) != 0) return fail(FMX_IO_ERR_OPEN, std::string("write failed: ") + path);
  return FMX_IO_OK;
}


const char* fmx_io_last_error(void) { return g_err.c_str(); }

int fmx_parse_double(const char* s, int64_t len, double* out) {
  if (!s || len < 0 || !out) return 0;
  return parse_value(std::string_view(s, size_t(len)), out) ? 1 : 0;
}

int fmx_csv_open(const char* path, const char* date_col, const char* symbol_col, int nthreads, fmx_csv** out) {
  if (!path || !date_col || !out) return fail(FMX_IO_ERR_ARG, "null argument");
  *out = nullptr;
  auto h = new fmx_csv();
  int fd = open(path, O_RDONLY);
  if (fd < 0) {
    delete h;
    return fail(FMX_IO_ERR_OPEN, std::string("cannot open ") + path + ": " + strerror(errno));
  }
  struct stat st;
  fstat(fd, &st);
  h->map_len = size_t(st.st_size);
  const char* b = "";
  if (h->map_len) {
    h->map = mmap(nullptr, h->map_len, PROT_READ, MAP_PRIVATE, fd, 0);
    if (h->map == MAP_FAILED) {
      close(fd);
      delete h;
      return fail(FMX_IO_ERR_OPEN, std::string("mmap failed: ") + strerror(errno));
    }
    madvise(h->map, h->map_len, MADV_SEQUENTIAL);
    b = static_cast<const char*>(h->map);
  }
  close(fd);
  const char* e = b + h->map_len;
  const char* nl = static_cast<const char*>(memchr(b, '\n', h->map_len));
  const char* he = nl ? nl : e;
  const char* body = nl ? nl + 1 : e;
  if (he > b && he[-1] == '\r') --he;
  if (he == b) {
    delete h;
    return fail(FMX_IO_ERR_FORMAT, "empty file or empty header line");
  }
  std::vector<std::string> cols;
  for (const char* q = b;;) {
    const char* comma = static_cast<const char*>(memchr(q, ',', size_t(he - q)));
    const char* fe = comma ? comma : he;
    cols.emplace_back(q, size_t(fe - q));
    if (!comma) break;
    q = comma + 1;
  }
  int dcol = -1, scol = -1;
  const bool has_sym = symbol_col && *symbol_col;
  for (int j = 0; j < int(cols.size()); ++j) {
    if (cols[j].find('"') != std::string::npos) {
      delete h;
      return fail(FMX_IO_ERR_FORMAT, "quoted header fields are not supported");
    }
    for (int i = 0; i < j; ++i)
      if (cols[i] == cols[j]) {   // pandas renames the second to 'x.1': not mirrored
        delete h;
        return fail(FMX_IO_ERR_FORMAT, "duplicate header name '" + cols[j] + "' is not supported");
      }
    if (cols[j] == date_col && dcol < 0) dcol = j;
    else if (has_sym && cols[j] == symbol_col && scol < 0) scol = j;
  }
  if (dcol < 0 || (has_sym && scol < 0)) {
    delete h;
    return fail(FMX_IO_ERR_FORMAT, std::string("header lacks column '") + (dcol < 0 ? date_col : symbol_col) + "'");
  }
  for (int j = 0; j < int(cols.size()); ++j)
    if (j != dcol && j != scol) h->names.push_back(cols[j]);
  const int ncol = int(cols.size());
  const int F = int(h->names.size());
  h->F = F;

  // newline-aligned chunks
  const int nt = pick_threads(nthreads);
  const int64_t body_len = int64_t(e - body);
  const int nchunk = int(std::max<int64_t>(1, std::min<int64_t>(nt * 4, body_len / (1 << 16) + 1)));
  h->chunks.resize(nchunk);
  const char* prev = body;
  for (int k = 0; k < nchunk; ++k) {
    const char* cut = (k == nchunk - 1) ? e : body + body_len * (k + 1) / nchunk;
    if (cut < prev) cut = prev;
    if (cut < e && k < nchunk - 1) {
      const char* n2 = static_cast<const char*>(memchr(cut, '\n', size_t(e - cut)));
      cut = n2 ? n2 + 1 : e;
    }
    h->chunks[k].b = prev;
    h->chunks[k].e = cut;
    prev = cut;
  }
  parallel_for(nt, nchunk, [&](int, int64_t lo, int64_t hi) {
    for (int64_t k = lo; k < hi; ++k) parse_chunk(h->chunks[k], ncol, dcol, scol, F);
  });
  int64_t rows = 0;
  for (auto& c : h->chunks) {
    if (!c.err.empty()) {
      std::string m = c.err;
      // chunk-local row numbers -> file-global
      size_t at = m.find(':');
      int64_t local = std::atoll(m.c_str() + 9);
      m = "data row " + std::to_string(rows + local) + m.substr(at);
      delete h;
      return fail(FMX_IO_ERR_FORMAT, m);
    }
    h->chunk_row0.push_back(rows);
    rows += c.rows;
  }
  h->n_rows = rows;
  h->int_cols.assign(F, rows > 0 ? 1 : 0);
  for (auto& c : h->chunks)
    for (int v = 0; v < F; ++v)
      if (c.not_int[v]) h->int_cols[v] = 0;

  // distinct dates and symbols, sorted
  std::vector<std::vector<int64_t>> ud(nchunk);
  std::vector<std::unordered_set<std::string_view>> us(nchunk);
  parallel_for(nt, nchunk, [&](int, int64_t lo, int64_t hi) {
    for (int64_t k = lo; k < hi; ++k) {
      auto& c = h->chunks[k];
      ud[k] = c.date_ns;
      std::sort(ud[k].begin(), ud[k].end());
      ud[k].erase(std::unique(ud[k].begin(), ud[k].end()), ud[k].end());
      us[k].insert(c.sym.begin(), c.sym.end());
    }
  });
  for (auto& v : ud) h->dates.insert(h->dates.end(), v.begin(), v.end());
  std::sort(h->dates.begin(), h->dates.end());
  h->dates.erase(std::unique(h->dates.begin(), h->dates.end()), h->dates.end());
  {
    std::unordered_set<std::string_view> all;
    for (auto& s : us) all.insert(s.begin(), s.end());
    h->symbols.assign(all.begin(), all.end());
    std::sort(h->symbols.begin(), h->symbols.end());
  }
  h->D = int64_t(h->dates.size());
  h->A = int64_t(h->symbols.size());
  std::unordered_map<std::string_view, int64_t> sidx;
  sidx.reserve(h->symbols.size() * 2);
  for (int64_t s = 0; s < h->A; ++s) sidx.emplace(h->symbols[s], s);

  h->flat.resize(rows);
  parallel_for(nt, nchunk, [&](int, int64_t lo, int64_t hi) {
    for (int64_t k = lo; k < hi; ++k) {
      auto& c = h->chunks[k];
      int64_t* fl = h->flat.data() + h->chunk_row0[k];
      for (int64_t r = 0; r < c.rows; ++r) {
        int64_t d = std::lower_bound(h->dates.begin(), h->dates.end(), c.date_ns[r]) - h->dates.begin();
        fl[r] = d * h->A + sidx.find(c.sym[r])->second;
      }
    }
  });
  // row-based semantics check (each symbol's rows in date order) + duplicate pairs
  {
    std::vector<int64_t> last(h->A, -1);
    std::vector<uint8_t> seen(size_t(h->D * h->A), 0);
    for (int64_t r = 0; r < rows; ++r) {
      const int64_t fl = h->flat[r], s = fl % h->A, d = fl / h->A;
      if (seen[fl] && h->dup_row < 0) h->dup_row = r;
      seen[fl] = 1;
      if (d <= last[s]) h->per_symbol_sorted = 0;
      last[s] = d;
    }
  }
  *out = h;
  return FMX_IO_OK;
}

int fmx_csv_close(fmx_csv* h) {
  delete h;
  return FMX_IO_OK;
}

int fmx_csv_shape(const fmx_csv* h, int64_t* n_rows, int64_t* n_values, int64_t* n_dates, int64_t* n_symbols,
                  int32_t* per_symbol_sorted) {
  if (!h) return fail(FMX_IO_ERR_ARG, "null handle");
  if (n_rows) *n_rows = h->n_rows;
  if (n_values) *n_values = h->F;
  if (n_dates) *n_dates = h->D;
  if (n_symbols) *n_symbols = h->A;
  if (per_symbol_sorted) *per_symbol_sorted = h->per_symbol_sorted;
  return FMX_IO_OK;
}

int fmx_csv_strings(const fmx_csv* h, int32_t which, char* buf, int64_t cap, int64_t* need) {
  if (!h || !need || (which != 0 && which != 1)) return fail(FMX_IO_ERR_ARG, "bad argument");
  std::string s;
  if (which == 0)
    for (auto& n : h->names) (s += n) += '\n';
  else
    for (auto& n : h->symbols) (s.append(n.data(), n.size())) += '\n';
  *need = int64_t(s.size());
  if (cap > 0) {
    if (!buf || cap < *need) return fail(FMX_IO_ERR_ARG, "buffer too small");
    memcpy(buf, s.data(), s.size());
  }
  return FMX_IO_OK;
}

int fmx_csv_dates(const fmx_csv* h, int64_t* ns) {
  if (!h || (!ns && h->D)) return fail(FMX_IO_ERR_ARG, "null argument");
  std::copy(h->dates.begin(), h->dates.end(), ns);
  return FMX_IO_OK;
}

int fmx_csv_rows(const fmx_csv* h, int64_t* flat) {
  if (!h || (!flat && h->n_rows)) return fail(FMX_IO_ERR_ARG, "null argument");
  std::copy(h->flat.begin(), h->flat.end(), flat);
  return FMX_IO_OK;
}

int fmx_csv_int_columns(const fmx_csv* h, int32_t* flags) {
  if (!h || (!flags && h->F)) return fail(FMX_IO_ERR_ARG, "null argument");
  std::copy(h->int_cols.begin(), h->int_cols.end(), flags);
  return FMX_IO_OK;
}

int fmx_csv_values(const fmx_csv* h, double* out, int nthreads) {
  if (!h || (!out && h->n_rows * h->F != 0)) return fail(FMX_IO_ERR_ARG, "null argument");
  const int64_t nchunk = int64_t(h->chunks.size());
  parallel_for(pick_threads(nthreads), nchunk, [&](int, int64_t lo, int64_t hi) {
    for (int64_t k = lo; k < hi; ++k) {
      auto& c = h->chunks[k];
      std::copy(c.vals.begin(), c.vals.end(), out + h->chunk_row0[k] * h->F);
    }
  });
  return FMX_IO_OK;
}

int fmx_csv_dense(const fmx_csv* h, double* out, int nthreads) {
  if (!h || (!out && h->F * h->D * h->A != 0)) return fail(FMX_IO_ERR_ARG, "null argument");
  if (h->dup_row >= 0)
    return fail(FMX_IO_ERR_DUPLICATE, "duplicate (date, symbol) pair at data row " + std::to_string(h->dup_row));
  const int nt = pick_threads(nthreads);
  const int64_t DA = h->D * h->A, F = h->F;
  if (h->n_rows < DA) {
    parallel_for(nt, F * DA, [&](int, int64_t lo, int64_t hi) { std::fill(out + lo, out + hi, double(NAN)); });
  }
  const int64_t nchunk = int64_t(h->chunks.size());
  parallel_for(nt, nchunk, [&](int, int64_t lo, int64_t hi) {
    for (int64_t k = lo; k < hi; ++k) {
      auto& c = h->chunks[k];
      const int64_t* fl = h->flat.data() + h->chunk_row0[k];
      // rows in tiles of 64 so each factor plane sees a run of nearby writes
      for (int64_t r0 = 0; r0 < c.rows; r0 += 64) {
        const int64_t r1 = std::min<int64_t>(c.rows, r0 + 64);
        for (int64_t f = 0; f < F; ++f) {
          double* plane = out + f * DA;
          const double* v = c.vals.data() + f;
          for (int64_t r = r0; r < r1; ++r) plane[fl[r]] = v[r * F];
        }
      }
    }
  });
  return FMX_IO_OK;
}

}  // extern "C"
