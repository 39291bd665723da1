// AddressSanitizer / UBSan driver of the host CSV loader (factormodeling_amd/csrc/csv_io.cpp,
// SURVEY.md §5 "Race detection / sanitizers"): test infrastructure, built by
// `make -C factormodeling_amd/csrc asan` into factormodeling_amd/csrc/build_asan/csv_asan
// and run by tests/test_csv_asan.py.  Every entry point of include/fmx_io.h is driven over
// the files named on the command line (mmap, multithreaded chunk parsing, sort, scatter,
// writer), plus the field parser over every line of a strings file.  Exit status 0 iff no
// call crashed; the sanitizers abort the process on the first memory / UB error.
//
//   csv_asan <strings.txt> <nthreads> <file.csv> <date_col> <symbol_col|-> [<file> <date> <sym>]...
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "../../include/fmx_io.h"

static int drive_file(const char* path, const char* date_col, const char* sym_col, int nt) {
  fmx_csv* h = nullptr;
  int st = fmx_csv_open(path, date_col, sym_col, nt, &h);
  if (st != FMX_IO_OK) {                        // format errors are expected for the bad files
    std::printf("open %s: status %d (%s)\n", path, st, fmx_io_last_error());
    return 0;
  }
  int64_t n_rows = 0, n_values = 0, D = 0, A = 0;
  int32_t sorted = 0;
  if (fmx_csv_shape(h, &n_rows, &n_values, &D, &A, &sorted)) return 1;
  std::vector<std::string> str(2);
  for (int which = 0; which < 2; ++which) {
    int64_t need = 0;
    fmx_csv_strings(h, which, nullptr, 0, &need);
    std::vector<char> buf((size_t)need + 1);
    if (fmx_csv_strings(h, which, buf.data(), need, &need)) return 1;
    str[which].assign(buf.data(), (size_t)need);
  }
  std::vector<int64_t> dates((size_t)D), flat((size_t)n_rows);
  std::vector<int32_t> ints((size_t)n_values);
  std::vector<double> vals((size_t)(n_rows * n_values)), dense((size_t)(n_values * D * A));
  if (fmx_csv_dates(h, dates.data()) || fmx_csv_rows(h, flat.data()) || fmx_csv_int_columns(h, ints.data()) ||
      fmx_csv_values(h, vals.data(), nt))
    return 1;
  st = fmx_csv_dense(h, dense.data(), nt);
  std::printf("file %s: rows %lld values %lld D %lld A %lld sorted %d dense %d\n", path, (long long)n_rows,
              (long long)n_values, (long long)D, (long long)A, sorted, st);
  if (st == FMX_IO_OK && n_values > 0) {
    // round trip through the writer: dates as their ns values, the loader's symbols
    std::string dstr;
    for (int64_t d = 0; d < D; ++d) dstr += std::to_string(dates[(size_t)d]) + "\n";
    std::vector<uint8_t> present((size_t)(D * A), 0);
    for (int64_t r = 0; r < n_rows; ++r) present[(size_t)flat[(size_t)r]] = 1;
    std::string hdr = "date,symbol";
    for (int64_t f = 0; f < n_values; ++f) hdr += ",v" + std::to_string(f);
    const std::string out = std::string(path) + ".asan_out.csv";
    const char* syms = (sym_col && *sym_col) ? str[1].c_str() : nullptr;
    if (syms || A == 1) {
      if (!syms) hdr = "date,v0";
      if (fmx_csv_write(out.c_str(), hdr.c_str(), dstr.c_str(), syms, dense.data(), syms ? n_values : 1, D, A,
                        present.data(), nt))
        std::printf("write %s: %s\n", out.c_str(), fmx_io_last_error());
    }
  }
  return fmx_csv_close(h);
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s strings.txt nthreads [file date_col symbol_col|-]...\n", argv[0]);
    return 2;
  }
  std::ifstream in(argv[1]);
  std::string line;
  char buf[64];
  long n = 0;
  while (std::getline(in, line)) {               // parser + formatter over every field
    double v = 0.0;
    fmx_parse_double(line.data(), (int64_t)line.size(), &v);
    if (fmx_format_double(v, buf, (int32_t)sizeof(buf)) < 0) return 1;
    ++n;
  }
  std::printf("fields %ld\n", n);
  const int nt = std::atoi(argv[2]);
  for (int i = 3; i + 2 < argc; i += 3) {
    const char* sym = std::strcmp(argv[i + 2], "-") == 0 ? "" : argv[i + 2];
    if (drive_file(argv[i], argv[i + 1], sym, nt)) {
      std::fprintf(stderr, "call failed on %s: %s\n", argv[i], fmx_io_last_error());
      return 1;
    }
  }
  std::printf("asan driver ok\n");
  return 0;
}
