/* fmx_io.h -- host-side C ABI of libfmx_io.so: the long-format CSV loader in front of the
 * factor-panel path.
 *
 * Replaces, in the reference notebook (pipeline.ipynb:71-82):
 *     df = pd.read_csv(path); df['date'] = pd.to_datetime(df['date'])
 *     df.set_index(['date', 'symbol'], inplace=True)
 * for the long files 2.symbol_features_long.csv / 8.factors_df.csv (one row per
 * (date, symbol), value columns after the keys) and, with no symbol column, the wide
 * 9.single_factor_returns.csv (one row per date).
 *
 * Semantics reproduced (pandas 2.3.3 C parser, the reference's loader):
 *   - value fields are parsed by a restatement of pandas' default float parser
 *     (tokenizer.c precise_xstrtod: 17 significant digits accumulated in a double, then
 *     one multiply/divide by a power-of-ten table) -- NOT correctly rounded, and
 *     bit-identical to pd.read_csv's default float_precision;
 *   - pandas' default NA strings ('', 'NaN', 'nan', 'NA', 'N/A', 'NULL', 'null', 'None',
 *     '<NA>', '#N/A', ...) give NaN; 'inf'/'-inf'/'infinity' (any case) give +-inf;
 *   - a column whose every field is an integer literal is flagged (pandas reads it as
 *     int64);
 *   - dates: ISO 'YYYY-MM-DD' optionally followed by ' HH:MM:SS[.fffffffff]' or 'T...',
 *     converted to nanoseconds since 1970-01-01 (pd.to_datetime).
 * Unsupported inputs (quoted fields, other date formats, non-numeric value fields, ragged
 * lines) return FMX_IO_ERR_FORMAT with a message naming the line; nothing is guessed.
 *
 * Threading: fmx_csv_open parses with `nthreads` host threads; a handle is read-only after
 * open and may be queried from any thread.  Errors: every call returns a status;
 * fmx_io_last_error() gives a thread-local message.
 */
#ifndef FMX_IO_H_
#define FMX_IO_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FMX_IO_OK 0
#define FMX_IO_ERR_ARG 1
#define FMX_IO_ERR_OPEN 2
#define FMX_IO_ERR_FORMAT 3
#define FMX_IO_ERR_DUPLICATE 4

typedef struct fmx_csv fmx_csv;

const char* fmx_io_last_error(void);

/* pandas tokenizer.c precise_xstrtod restated over [s, s+len): value into *out, returns 1
 * when the whole field (after optional surrounding blanks) was consumed, else 0.  Exposed
 * for the parity tests. */
int fmx_parse_double(const char* s, int64_t len, double* out);

/* Parse a whole file.  date_col must name a column; symbol_col may be NULL or "" (wide
 * files indexed by date only: one symbol). */
int fmx_csv_open(const char* path, const char* date_col, const char* symbol_col, int nthreads,
                 fmx_csv** out);
int fmx_csv_close(fmx_csv* h);

/* n_rows data rows, n_values value columns, D distinct dates, A distinct symbols;
 * *per_symbol_sorted = 1 iff every symbol's rows appear in increasing date order. */
int fmx_csv_shape(const fmx_csv* h, int64_t* n_rows, int64_t* n_values, int64_t* n_dates,
                  int64_t* n_symbols, int32_t* per_symbol_sorted);
/* Value column names, then sorted distinct symbols (byte order), each '\n'-terminated,
 * into buf[cap]; *need = bytes required (call with cap 0 to size). which: 0 names,
 * 1 symbols. */
int fmx_csv_strings(const fmx_csv* h, int32_t which, char* buf, int64_t cap, int64_t* need);
/* Sorted distinct dates, ns since epoch [D]. */
int fmx_csv_dates(const fmx_csv* h, int64_t* ns);
/* Per data row (file order): d * A + s  [n_rows]. */
int fmx_csv_rows(const fmx_csv* h, int64_t* flat);
/* Per value column: 1 iff every field is an integer literal (pandas int64 column). */
int fmx_csv_int_columns(const fmx_csv* h, int32_t* flags);
/* Row-major values in file order [n_rows][n_values]. */
int fmx_csv_values(const fmx_csv* h, double* out, int nthreads);
/* Dense panel [n_values][D][A] (the engine's X layout), NaN where a (date, symbol) row is
 * absent; fails with FMX_IO_ERR_DUPLICATE if a (date, symbol) pair repeats. */
int fmx_csv_dense(const fmx_csv* h, double* out, int nthreads);

/* Writer for the checkpoint CSVs the notebook emits with DataFrame/Series.to_csv
 * (pipeline.ipynb:217,364,391,420,464-466): `header` line, then one row per present
 * (date, symbol) cell in date-major order: date string, symbol string (omitted when
 * symbol_strs is NULL, then A must be 1), and X[f][d][a] for f < F formatted like Python
 * repr(float) (pandas' float64 cells; NaN -> empty).  date_strs / symbol_strs hold D / A
 * '\n'-terminated strings.  present [D][A] may be NULL (all cells). */
int fmx_csv_write(const char* path, const char* header, const char* date_strs, const char* symbol_strs,
                  const double* X, int64_t F, int64_t D, int64_t A, const uint8_t* present, int nthreads);
/* repr(float) of x into buf (NUL-terminated); returns its length, -1 if cap is too small. */
int fmx_format_double(double x, char* buf, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* FMX_IO_H_ */
