/*
 * fmx.h -- C ABI of libfmx, the MI355X (gfx950) engine for the FactorModeling
 * factor-panel hot path.
 *
 * Boundary: the reference (Yuming-Yang/FactorModeling) is pure Python; its "FFI" for this
 * path is the set of Python functions in operations.py, factor_selector.py,
 * factor_selection_methods.py and composite_factor.py.  The drop-in modules in
 * factormodeling_amd/ keep those signatures and bind the entry points below through
 * ctypes.  Each entry point names the reference function(s) it
 * replaces.
 *
 * Conventions
 *   - Panels are device pointers to float64 X[F][D][ld] (factor, date, asset; asset
 *     fastest; ld >= A is the row stride in elements).  Returns R are [D][ld].
 *   - present: optional device uint8[D][ld]; 0 marks a (date, symbol) pair with no row
 *     in the reference's long (date, symbol) MultiIndex.  NULL = dense panel.
 *     Time-series ops walk each symbol's present rows (row-based, as the reference's
 *     groupby('symbol') + rolling/shift); cross-sectional ops reduce over the present
 *     rows of a date.  Outputs at absent cells are NaN.
 *   - stream: a hipStream_t passed as void* (NULL = default stream).  All calls are
 *     stream-ordered and asynchronous; no call allocates on the hot path (the only
 *     hipMalloc is the one-time cache of a row length's pairwise-sum schedule).
 *   - Scratch: calls that need device scratch take (work, work_bytes) from the caller,
 *     sized by the matching fmx_*_work_bytes / fmx_*_work_len query; one buffer may be
 *     reused by every call on the same stream.
 *   - Errors: every call returns an fmx_status; fmx_last_error() gives a thread-local
 *     message.  No exceptions cross the ABI.
 */
#ifndef FMX_H_
#define FMX_H_

#include <stdint.h>

/* Doubled average rank of a cell among its row's non-NaN cells (2*#less + #equal + 1; 0
 * for NaN): <= 2A <= 32768 for the A <= 16384 rows the ranked kernels take, so 16 bits. */
typedef uint16_t fmx_rank2_t;

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t fmx_status;
#define FMX_OK 0
#define FMX_ERR_ARG 1
#define FMX_ERR_HIP 2
#define FMX_ERR_UNSUPPORTED 3
#define FMX_ERR_NOMEM 4

#define FMX_ABI_VERSION 1

/* time-series ops (fmx_ts_op) */
#define FMX_TS_SUM 0      /* operations.py:6   ts_sum      rolling(w).sum()            */
#define FMX_TS_MEAN 1     /* operations.py:10  ts_mean     rolling(w).mean()           */
#define FMX_TS_STD 2      /* operations.py:14  ts_std      rolling(w).std()            */
#define FMX_TS_VAR 3      /*                   rolling(w).var() (helper)               */
#define FMX_TS_ZSCORE 4   /* operations.py:18  ts_zscore                               */
#define FMX_TS_RANK 5     /* operations.py:23  ts_rank     pct rank of last in window  */
#define FMX_TS_DECAY 6    /* operations.py:40  ts_decay    linear-weight MA            */
#define FMX_TS_DIFF 7     /* operations.py:34  ts_diff     diff(w), w may be <= 0      */
#define FMX_TS_DELAY 8    /* operations.py:37  ts_delay    shift(w), w may be <= 0     */
#define FMX_TS_BACKFILL 9 /* operations.py:50  ts_backfill ffill()                     */

/* cross-sectional moment ops (fmx_cs_moment) */
#define FMX_CS_ZSCORE 0            /* operations.py:77  cs_zscore         */
#define FMX_CS_MEAN 1              /* operations.py:85  cs_mean           */
#define FMX_CS_MARKET_NEUTRALIZE 2 /* operations.py:171 market_neutralize */
#define FMX_CS_STATS 3             /* row (mean, std ddof=0) only (fmx_cs_moment_stats) */

/* rank methods (pandas Series.rank(method=...)) */
#define FMX_RANK_AVERAGE 0
#define FMX_RANK_MIN 1
#define FMX_RANK_MAX 2
#define FMX_RANK_FIRST 3
#define FMX_RANK_DENSE 4
#define FMX_RANK_AVERAGE_PROPAGATE 5 /* scipy.stats.rankdata: any NaN -> row NaN; no 0.5 rule */

/* group ops (fmx_group_op) */
#define FMX_GROUP_MEAN 0       /* operations.py:112 group_mean            */
#define FMX_GROUP_NEUTRALIZE 1 /* operations.py:124 group_neutralize      */
#define FMX_GROUP_NORMALIZE 2  /* operations.py:137 group_normalize       */
#define FMX_GROUP_RANK 3       /* operations.py:152 group_rank_normalized */

/* elementwise ops (fmx_elementwise) */
#define FMX_EW_SIGN 0  /* operations.py:88  sign            */
#define FMX_EW_POWER 1 /* operations.py:91  power(x, a)     */
#define FMX_EW_LOG 2   /* operations.py:94  log             */
#define FMX_EW_ABS 3   /* operations.py:97  abs_            */
#define FMX_EW_CLIP 4  /* operations.py:100 clip(x, a, b)   */
#define FMX_EW_WHERE 5 /* operations.py:80  cs_bool(cond, a, b), cond as 0/1 */

/* cs_regression rettype (operations.py:248) */
#define FMX_CSREG_RESID 0
#define FMX_CSREG_BETA 1
#define FMX_CSREG_ALPHA 2
#define FMX_CSREG_FITTED 3
#define FMX_CSREG_R2 4

/* ---- library ------------------------------------------------------------------ */
const char* fmx_last_error(void);
int32_t fmx_abi_version(void);
/* "product", or "diagnostic: ..." for a development build whose kernels carry wrong-result
 * timing arms (-DFMX_DIAG); the Python loader refuses the latter unless FMX_ALLOW_DIAG=1. */
const char* fmx_build_variant(void);
/* Writes "gfx950 ... CUs ... HBM bytes" of the current device into buf. */
fmx_status fmx_device_info(char* buf, int64_t buflen);

/* ---- time series (operations.py:6-51) -------------------------------------------- */
/* Replaces ts_sum/ts_mean/ts_std/ts_zscore/ts_rank/ts_decay/ts_diff/ts_delay/ts_backfill
 * (operations.py:6-51).  Y may not alias X.  Rolling sums/means/variances reproduce
 * pandas' Kahan/Welford kernels bit-for-bit.  Any window (no LDS ring: DESIGN §12), dense
 * or ragged; window < 0 for diff / delay is a lead. */
fmx_status fmx_ts_op(int32_t op, const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                     int32_t window, const uint8_t* present, void* stream);

/* Fused rolling set: ts_mean(window), ts_std(window), ts_zscore(window), ts_rank(rank_window)
 * and ts_decay(window) (operations.py:10-48) from ONE read of X.  Any output may be NULL
 * (not computed); none may alias X.  Each output is bit-identical to fmx_ts_op of that op.
 * Dense panels with (window, rank_window) = (20, 10) run one fused kernel; other windows
 * and ragged panels run one fmx_ts_op pass per requested output. */
fmx_status fmx_ts_set(const double* X, double* Ymean, double* Ystd, double* Yzscore, double* Yrank, double* Ydecay,
                      int64_t F, int64_t D, int64_t A, int64_t ld, int32_t window, int32_t rank_window,
                      const uint8_t* present, void* stream);

/* Builder-defined ts_corr (no reference counterpart): per-symbol rolling Pearson of X[f]
 * against Ycol (y_fstride = 0: one [D][ld] series shared by all factors, e.g. returns),
 * pandas Rolling.corr semantics, min_periods = window. */
fmx_status fmx_ts_corr(const double* X, const double* Ycol, double* Out, int64_t F, int64_t D, int64_t A,
                       int64_t ld, int64_t y_fstride, int32_t window, const uint8_t* present, void* stream);

/* ts_regression_fast rolling moments (operations.py:185-246) for one [D][ld] pair.
 * Xv is the globally shifted x; valid marks rows kept by the reference's dropna().
 * rettype 0 resid, 1 alpha, 2 beta, 3 fitted, 6 R^2.  NaN where not computed. */
fmx_status fmx_ts_regression(const double* Yv, const double* Xv, const uint8_t* valid, double* Out, int64_t D,
                             int64_t A, int64_t ld, int32_t window, int32_t rettype, void* stream);

/* ---- cross section (operations.py:54-101, 171-182, 248-304) ---------------------- */
fmx_status fmx_cs_moment(int32_t op, const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                         const uint8_t* present, void* stream);
/* fmx_cs_moment that also writes stats[F][D][2] = (nanmean, nanstd ddof=0) per row, the
 * numpy-pairwise moments cs_zscore uses (operations.py:77-78).  op FMX_CS_STATS writes
 * only the stats (Y may be NULL); they feed fmx_gram_fused. */
fmx_status fmx_cs_moment_stats(int32_t op, const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                               const uint8_t* present, double* stats, void* stream);

/* C5's feature (builder-defined; BASELINE configs[4] "60-day rolling ts_corr/ts_std feeding
 * IC-weighted composite"): Y = sign(C) * (X / ts_std(X, window)) per column, ts_std ==
 * 0 -> NaN, C = fmx_ts_corr(X, R, window) of the same rows (np.sign semantics).  The std is
 * pandas' rolling Welford (operations.py:14-15), bit-identical to fmx_ts_op(FMX_TS_STD).
 * Dense panels. */
fmx_status fmx_ts_corr_vol_feature(const double* X, const double* C, double* Y, int64_t F, int64_t D, int64_t A,
                                   int64_t ld, int32_t window, void* stream);
/* The same feature straight from the returns in ONE pass (C5's chain: ts_corr of x with
 * Ycol feeding sign(corr) * x / ts_std(x, window), pipeline.ipynb's corr-vol signal): the
 * corr panel is neither written nor re-read.  Y is bit-identical to fmx_ts_corr (dense) +
 * fmx_ts_corr_vol_feature; C, when not NULL, also receives the corr.  Dense panels,
 * 1 <= window <= 4096, Ycol as in fmx_ts_corr (y_fstride 0: one [D][ld] return panel). */
fmx_status fmx_ts_corr_feature(const double* X, const double* Ycol, double* C, double* Y, int64_t F, int64_t D,
                               int64_t A, int64_t ld, int64_t y_fstride, int32_t window, void* stream);
/* cs_zscore (Yz) and market_neutralize (Yn) of the same rows from ONE set of moments
 * (operations.py:77-78, :171-182); optional stats[F][D][2] = (mean, std ddof=0).  Outputs
 * bit-identical to fmx_cs_moment of each op; distinct from X and each other. */
fmx_status fmx_cs_zscore_neutralize(const double* X, double* Yz, double* Yn, int64_t F, int64_t D, int64_t A,
                                    int64_t ld, const uint8_t* present, double* stats, void* stream);
/* cs_rank (operations.py:54-62): (rank - 1) / (rows - 1), rows counting NaN. */
fmx_status fmx_cs_rank(const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld, int32_t method,
                       const uint8_t* present, void* stream);

/* cs_rank(method='average') and cs_winsor(limits=(qlo, qhi)) of the same rows in ONE pass
 * (operations.py:54-68): the winsor quantiles' order statistics are read off the rank
 * histogram.  Outputs bit-identical to fmx_cs_rank / fmx_cs_winsor; distinct from X.
 * rank2 (optional, device fmx_rank2_t [F][D][ld], needs present == NULL and A <= 16384): the
 * doubled average rank of every non-NaN cell (2*#less + #equal + 1; 0 for NaN), the input
 * of fmx_ic_daily_ranked. */
fmx_status fmx_cs_rank_winsor(const double* X, double* Yrank, double* Ywinsor, int64_t F, int64_t D, int64_t A,
                              int64_t ld, double qlo, double qhi, const uint8_t* present, fmx_rank2_t* rank2,
                              void* stream);
/* cs_rank (average) + cs_winsor (qlo, qhi) + cs_zscore + market_neutralize of the same dense
 * rows in ONE pass (operations.py:54-68, :77-78, :171-182): each row is read once for the
 * four operators; every output is bit-identical to its own entry point (fmx_cs_rank_winsor,
 * fmx_cs_zscore_neutralize); rank2 as in fmx_cs_rank_winsor (or NULL).  Five distinct
 * panels.  Rows past the fused kernel (A > 16384) take the two two-output passes. */
fmx_status fmx_cs_rank_winsor_zn(const double* X, double* Yrank, double* Ywinsor, double* Yzscore, double* Yneutralize,
                                 int64_t F, int64_t D, int64_t A, int64_t ld, double qlo, double qhi,
                                 fmx_rank2_t* rank2, void* stream);
/* cs_rank, every method, for any row length (A <= 65535): rows sorted in HBM (rocPRIM
 * segmented radix sort of (value key, asset) pairs, stable), then one wave per row walks
 * its tie runs and scatters the ranks.  fmx_cs_rank takes 'first' / 'dense' up to A = 8192
 * (LDS bitonic) and the other methods up to 16384 (fine buckets); this entry has no such
 * limit.  work: fmx_cs_rank_sorted_work_bytes(F, D, A). */
fmx_status fmx_cs_rank_sorted(const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld, int32_t method,
                              const uint8_t* present, void* work, int64_t work_bytes, void* stream);
int64_t fmx_cs_rank_sorted_work_bytes(int64_t F, int64_t D, int64_t A);
/* cs_winsor (op 0) / cs_filter_center (op 1) (operations.py:64-75) for any row length
 * (A <= 65535): the numpy 'linear' order statistics read off the sorted rows.  work:
 * fmx_cs_rank_sorted_work_bytes(F, D, A). */
fmx_status fmx_cs_quantile_sorted(int32_t op, const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                                  double qlo, double qhi, const uint8_t* present, void* work, int64_t work_bytes,
                                  void* stream);
/* group_rank_normalized (operations.py:152-168) for any group size and row length (A <=
 * 65535): rows sorted by (group, value) in two stable passes.  G, ngroups as fmx_group_op;
 * methods average / min / max / first / dense.  work: fmx_group_rank_sorted_work_bytes. */
fmx_status fmx_group_rank_sorted(const double* X, const int32_t* G, double* Y, int64_t F, int64_t D, int64_t A,
                                 int64_t ld, int32_t ngroups, int32_t method, const uint8_t* present, void* work,
                                 int64_t work_bytes, void* stream);
int64_t fmx_group_rank_sorted_work_bytes(int64_t F, int64_t D, int64_t A);
/* Only the doubled average ranks of fmx_cs_rank_winsor (rank2 [F][D][ld] fmx_rank2_t, A <=
 * 16384): the rank pass of a daily IC over raw factors (fmx_ic_daily_ranked) when no
 * operator output of the same rows is wanted (factor_selector.py:36-48's rankdata). */
fmx_status fmx_cs_rank2(const double* X, fmx_rank2_t* rank2, int64_t F, int64_t D, int64_t A, int64_t ld,
                        void* stream);
/* fmx_cs_rank_winsor_zn / fmx_cs_rank2 on the rows of dates [d0, d1) of every factor of an
 * [F][D][ld] panel (outputs at the same rows; other rows untouched).  The date-sharded step
 * runs the four operators on its owned dates while the halo exchange is in flight and the
 * doubled ranks of the halo rows after it (the daily IC reads exposures at t - lag).
 * Replaces the same reference functions as the two whole-panel entries
 * (operations.py:54-68, :77-78, :171-182; factor_selector.py:36-48).  A <= 16384. */
fmx_status fmx_cs_rank_winsor_zn_dates(const double* X, double* Yrank, double* Ywinsor, double* Yzscore,
                                       double* Yneutralize, int64_t F, int64_t D, int64_t A, int64_t ld, int64_t d0,
                                       int64_t d1, double qlo, double qhi, fmx_rank2_t* rank2, void* stream);
fmx_status fmx_cs_rank2_dates(const double* X, fmx_rank2_t* rank2, int64_t F, int64_t D, int64_t A, int64_t ld,
                              int64_t d0, int64_t d1, void* stream);
/* cs_winsor (operations.py:64-68); qlo/qhi are the fractions numpy sees
 * (pandas passes q*100 and numpy divides by 100). */
fmx_status fmx_cs_winsor(const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld, double qlo,
                         double qhi, const uint8_t* present, void* stream);
/* cs_filter_center (operations.py:70-75). */
fmx_status fmx_cs_filter_center(const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                                double qlo, double qhi, const uint8_t* present, void* stream);
/* group ops (operations.py:112-168).  G: device int32[D][ld] dense group ids, -1 = NaN.
 * Rows up to 4096 assets: whole-row LDS sort; up to 16384: per-group compaction (the rank
 * sorts each group in LDS: groups of <= 8192 members, larger groups come out NaN --
 * factormodeling_amd.engine.group_op checks and raises before the launch).  Rank methods
 * average / min / max / first / dense. */
fmx_status fmx_group_op(int32_t op, const double* X, const int32_t* G, double* Y, int64_t F, int64_t D, int64_t A,
                        int64_t ld, int32_t ngroups, int32_t method, const uint8_t* present, void* stream);
/* group_mean / group_neutralize / group_normalize (operations.py:112-149) on rows of ANY
 * length up to 65,535 assets (fmx_group_op holds a row in registers: A <= 16384): rows
 * stay in HBM, each group's members are compacted in asset order into device scratch and
 * summed with numpy's pairwise schedule (bit-identical to fmx_group_op where both run).
 * Codes outside [0, ngroups) = no group.  work: fmx_group_op_long_work_bytes(F, D, A). */
int64_t fmx_group_op_long_work_bytes(int64_t F, int64_t D, int64_t A);
fmx_status fmx_group_op_long(int32_t op, const double* X, const int32_t* G, double* Y, int64_t F, int64_t D, int64_t A,
                             int64_t ld, int32_t ngroups, const uint8_t* present, void* work, int64_t work_bytes,
                             void* stream);
/* cs_regression (operations.py:248-304) for one [D][ld] pair. */
fmx_status fmx_cs_regression(const double* Yv, const double* Xv, double* Out, int64_t D, int64_t A, int64_t ld,
                             int32_t rettype, const uint8_t* present, void* stream);
/* elementwise over n contiguous doubles (operations.py:80-101). */
fmx_status fmx_elementwise(int32_t op, const double* X, double* Y, int64_t n, double a, double b, void* stream);
/* bucket (operations.py:104-110): pd.cut(right=True, include_lowest=True) label codes. */
fmx_status fmx_bucket(const double* X, int32_t* codes, int64_t n, const double* edges, int32_t n_edges,
                      void* stream);

/* ---- IC, metrics, selection (factor_selector.py:26-139, factor_selection_methods.py:6-26) */
/* Daily stats for each lag in lags[0..n_lags) (HOST int32 array, lags >= 0): pairs
 * (X[f][t-L], R[t]).  out: [n_lags][4][F][D] = (n_pairs, IC, rank_IC, beta); NaN where
 * undefined.  Each exposure row is ranked once for up to two lags. */
fmx_status fmx_ic_daily(const double* X, const double* R, int64_t F, int64_t D, int64_t A, int64_t ld,
                        const int32_t* lags, int32_t n_lags, double* out, void* stream);
/* Daily IC records for rows of ANY length up to 65,535 assets (the fine kernels' 16-bit
 * doubled ranks end at 16,384; factor_selector.py:36-48 has no limit): each (f, s) row
 * is sorted in HBM (rocPRIM segmented radix sort, chunks of rows), then one wave per row
 * ranks each lag's pair-valid subset off the sorted keys and reduces the same
 * (n, IC, rank IC, beta) records as fmx_ic_daily (out layout identical).  work:
 * fmx_ic_daily_sorted_work_bytes(F, D, A) bytes of device scratch. */
int64_t fmx_ic_daily_sorted_work_bytes(int64_t F, int64_t D, int64_t A);
fmx_status fmx_ic_daily_sorted(const double* X, const double* R, int64_t F, int64_t D, int64_t A, int64_t ld,
                               const int32_t* lags, int32_t n_lags, double* out, void* work, int64_t work_bytes,
                               void* stream);
/* fmx_ic_daily for a panel whose rows fmx_cs_rank_winsor already ranked (rank2): the
 * rank among each lag's pairs is rank2 corrected by the exposures whose return is NaN, so
 * no row is ranked again; one wavefront per row (single-pass shifted moments: records
 * agree with fmx_ic_daily to ~1e-15 relative, pair counts exactly).  work: device int32
 * scratch of fmx_ic_ranked_work_len(F, D) elements.  A <= 16384. */
int64_t fmx_ic_ranked_work_len(int64_t F, int64_t D);
fmx_status fmx_ic_daily_ranked(const double* X, const fmx_rank2_t* rank2, const double* R, int64_t F, int64_t D,
                               int64_t A, int64_t ld, const int32_t* lags, int32_t n_lags, int32_t* work,
                               int64_t work_len, double* out, void* stream);
/* cs_rank(method='average') + cs_winsor (operations.py:54-68) AND the daily IC of the same
 * rows (factor_selector.py:36-48: pearsonr, pearsonr(rankdata), beta of the pairs
 * (X[f][t-L], R[t])) in ONE pass: each row's ranks feed its IC records inside the
 * workgroup, so no rank panel is written or re-read.  Yrank / Ywinsor: both set (outputs
 * bit-identical to fmx_cs_rank_winsor) or both NULL (the IC's rank pass alone).  lags: HOST
 * int32[n_lags], n_lags 1 or 2; out as fmx_ic_daily (records agree with it to ~1e-15
 * relative, pair counts exactly).  rank2: device fmx_rank2_t [F][D][ld] scratch, written
 * only for rows with > 256 NaN returns (finished by the workgroup kernel of
 * fmx_ic_daily_ranked).  work: device int32 of fmx_rank_ic_work_len(F, D, A).  Dense rows
 * (no presence mask), A <= 16384. */
int64_t fmx_rank_ic_work_len(int64_t F, int64_t D, int64_t A);
fmx_status fmx_cs_rank_winsor_ic(const double* X, double* Yrank, double* Ywinsor, const double* R, int64_t F,
                                 int64_t D, int64_t A, int64_t ld, double qlo, double qhi, const int32_t* lags,
                                 int32_t n_lags, fmx_rank2_t* rank2, int32_t* work, int64_t work_len, double* out,
                                 void* stream);
/* Window summaries of one lag's daily stats [4][F][D] over J date windows [d0, d1).
 * out: [J][F][8] = IC, IC_IR, rank_IC, rank_IC_IR, tstat, n_beta, pct_pos, n_days. */
fmx_status fmx_ic_window(const double* daily, int64_t F, int64_t D, const int32_t* d0_dev, const int32_t* d1_dev,
                         int64_t J, double* out, void* stream);
/* icir_top_selector (factor_selection_methods.py:6-26) for J days of window metrics.
 * order_out [J][F] (rank_IC_IR-descending factor order), w_out [J][F] weights. */
fmx_status fmx_select_icir_top(const double* metrics, int64_t J, int64_t F, int32_t use_rank_icir,
                               double threshold, int32_t top_x, int32_t* order_out, double* w_out, void* stream);

/* ---- factor correlation GEMM (builder-defined) ------------------------ */
/* Z: per-date z-scored exposures (float64 [F][D][ld], NaN -> 0); M: validity as bf16
 * 0/1 (uint16 bit patterns [F][D][ld]).  stats: fmx_cs_moment_stats' [F][D][2] (mean, sd)
 * -- the oracle's numpy moments bit for bit -- or NULL for in-kernel block sums. */
fmx_status fmx_zscore_exposures(const double* X, const double* stats, double* Z, uint16_t* M, int64_t F, int64_t D,
                                int64_t A, int64_t ld, void* stream);
/* fmx_zscore_exposures for the dates [d0, d1) only: Z / M are [F][d1 - d0][ld] (chunked
 * Gram of a panel whose full Z / M would not fit next to X, e.g. C4 at 121 GB). */
fmx_status fmx_zscore_exposures_range(const double* X, const double* stats, double* Z, uint16_t* M, int64_t F,
                                      int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t d1, void* stream);
/* G[F][F] (+)= sum_{d in [d0,d1), a} Z[i][d][a] Z[j][d][a] on fp64 MFMA
 * (v_mfma_f64_16x16x4_f64) and N[F][F] (+)= the same sum over M on bf16 MFMA (exact
 * pair counts).  accumulate = 0 overwrites.  M/N may be NULL. */
/* The wide-panel correlation Gram straight from the raw panel (builder-defined A19, C4's
 * 2000 x 2000): G = Z^T Z (fp64 MFMA, 128 x 128 tiles) with Z z-scored while each tile
 * chunk is staged from stats[F][D][2] (fmx_cs_moment_stats: numpy-pairwise mean / std
 * ddof=0; NaN -> 0, sigma 0 or NaN -> row 0), and N = M^T M as AND + popcount of validity
 * bits (exact).  No Z / M panels are materialised.  Dates [d0, d1); accumulate adds into
 * G / N.  work: fmx_gram_direct_work_bytes. */
int64_t fmx_gram_direct_work_bytes(int64_t F, int64_t D, int64_t A, int64_t d0, int64_t d1);
fmx_status fmx_gram_direct(const double* X, const double* stats, double* G, double* N, int64_t F, int64_t D,
                           int64_t A, int64_t ld, int64_t d0, int64_t d1, int32_t accumulate, void* work,
                           int64_t work_bytes, void* stream);
fmx_status fmx_gram(const double* Z, const uint16_t* M, double* G, double* N, int64_t F, int64_t D, int64_t A,
                    int64_t ld, int64_t d0, int64_t d1, int32_t accumulate, void* work, int64_t work_bytes,
                    void* stream);
/* Device workspace fmx_gram needs for these dims (with_mask: M and N given). */
int64_t fmx_gram_work_bytes(int64_t F, int64_t D, int64_t A, int64_t d0, int64_t d1, int32_t with_mask);
/* Fused form for F <= 256: G and N straight from the raw panel X with the row stats of
 * fmx_cs_moment_stats (z = (x - mean) / sd where x is non-NaN and sd > 0, else 0; M the
 * same validity), one pass over X, both MFMA products in the same workgroup.  stats ==
 * NULL: X already holds the z-scores (the fmx_cs_zscore output of the same rows: z is
 * used where finite, else 0 / invalid -- the same Z and M).  Returns
 * FMX_ERR_UNSUPPORTED for F > 256 (use fmx_zscore_exposures + fmx_gram). */
fmx_status fmx_gram_fused(const double* X, const double* stats, double* G, double* N, int64_t F, int64_t D,
                          int64_t A, int64_t ld, int64_t d0, int64_t d1, int32_t accumulate, void* work,
                          int64_t work_bytes, void* stream);
/* Device workspace fmx_gram_fused needs (per-slice partial tiles, validity bits, counts). */
int64_t fmx_gram_fused_work_bytes(int64_t F, int64_t D, int64_t A, int64_t d0, int64_t d1);
/* Exact, GPU-count-independent form of fmx_gram_fused (F <= 256) for the date-sharded
 * step (SURVEY 5 "bit-identical at 1/2/4/8 GPUs"; replaces the float sum of Gram partials
 * behind the builder-defined corr-prune, A19).  The dates [d0, d1) are cut into fixed
 * units (fmx_gram_exact_units_per_date(A) asset ranges per date), each unit's Z^T Z is
 * computed on fp64 MFMA and folded into a signed fixed-point accumulator (LSB 2^-64, 6 x
 * 32-bit payload limbs in int64 + an invalid-term flag): limbs [FMX_GRAM_EXACT_SLOTS][F][F]
 * (upper triangle), counts [F][F] int64 pair counts (upper triangle).  Both are plain
 * integer sums, so ranks add them with an int64 all-reduce (any order) and
 * fmx_gram_exact_finalize gives the same G and N bits at every GPU count.  accumulate = 0
 * zeroes limbs and counts first.  stats == NULL: X holds the z-scores (as fmx_gram_fused). */
#define FMX_GRAM_EXACT_SLOTS 7
fmx_status fmx_gram_exact(const double* X, const double* stats, int64_t* limbs, int64_t* counts, int64_t F,
                          int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t d1, int32_t accumulate, void* work,
                          int64_t work_bytes, void* stream);
int64_t fmx_gram_exact_work_bytes(int64_t F, int64_t D, int64_t A, int64_t d0, int64_t d1);
/* Exact, GPU-count-independent form of fmx_gram_direct (any F; C4's 2000 x 2000 at
 * 2/4/8 GPUs, builder-defined A19).  The tile kernel's date slices are ABSOLUTE blocks of
 * FMX_GRAM_DATE_BLOCK dates (local row 0 of X is absolute date d_origin); each block's fp64
 * partial tiles fold into the same fixed-point limbs as fmx_gram_exact.  A date shard whose
 * bounds are multiples of FMX_GRAM_DATE_BLOCK holds whole blocks, so an int64 all-reduce of
 * limbs / counts + fmx_gram_exact_finalize gives the same G, N bits at every GPU count.
 * accumulate = 0 zeroes limbs and counts first.  work: fmx_gram_direct_exact_work_bytes.
 * Rows of 8..8192 assets (the default): a z pass computes the row moments itself, writes
 * zero-filled z-scores for chunks of 32 date blocks into the workspace and an LDS-DMA tile
 * kernel multiplies them, so stats is ignored and may be NULL.  Other rows (or
 * FMX_GRAM_ZC=0) z-score while staging from stats = fmx_cs_moment_stats (mean, std) [F][D][2];
 * NULL there computes them into the workspace first. */
#define FMX_GRAM_DATE_BLOCK 16
fmx_status fmx_gram_direct_exact(const double* X, const double* stats, int64_t* limbs, int64_t* counts, int64_t F,
                                 int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t d1, int64_t d_origin,
                                 int32_t accumulate, void* work, int64_t work_bytes, void* stream);
int64_t fmx_gram_direct_exact_work_bytes(int64_t F, int64_t D, int64_t A, int64_t d0, int64_t d1, int64_t d_origin);
/* G, N [F][F] (symmetric) from exact limbs / counts (N and counts may be NULL); a flagged
 * (non-finite or >= 2^127) term makes the entry NaN. */
fmx_status fmx_gram_exact_finalize(const int64_t* limbs, const int64_t* counts, double* G, double* N, int64_t F,
                                   void* stream);
int32_t fmx_gram_exact_units_per_date(int64_t A);
/* Host-side run of the same accumulator over n doubles (test hook; no GPU needed). */
void fmx_debug_exact_fold(const double* x, int64_t n, int64_t* limbs_out, double* value_out);
/* The step's greedy prune (builder-defined A19, the host walk of engine.greedy_prune): walk
 * order[0..n_order); factor f is kept iff max over the kept k of |C[f][k]| is NaN or < rho;
 * at most top_x kept.  C is the symmetric correlation matrix [F][ldc] on the device; kept
 * (int32 [top_x or F]) and n_kept (int32 [1]) are device buffers.  F <= 20480. */
fmx_status fmx_greedy_prune(const double* C, int64_t F, int64_t ldc, const int64_t* order, int64_t n_order,
                            double rho, int64_t top_x, int32_t* kept, int32_t* n_kept, void* stream);

/* The builder-defined corr_prune selector for J rolling windows in one call:
 * per-date Gram partials of the raw panel X (z-scored with stats [F][D][2] from
 * fmx_cs_moment_stats) for every date any window touches, then per window j the pooled
 * G / N over raw dates [s0_host[j], s0_host[j] + window) (the lag-1 factors of the window's
 * dates) and the greedy walk of order [J][F] (metrics [J][F][8] column rank_IC_IR or IC_IR
 * > threshold; keep iff |C| < rho against every kept factor; up to top_x).  w_out [J][F] =
 * 1 / #kept on the kept factors.  F <= 256. */
fmx_status fmx_corr_prune_windows(const double* X, const double* stats, int64_t F, int64_t D, int64_t A, int64_t ld,
                                  int64_t J, int32_t window, const int32_t* s0_host, const int32_t* order,
                                  const double* metrics, int32_t use_rank_icir, double threshold, double rho,
                                  int32_t top_x, double* w_out, void* work, int64_t work_bytes, void* stream);
/* Device workspace fmx_corr_prune_windows needs (per-date partials of the touched dates). */
int64_t fmx_corr_prune_windows_work_bytes(int64_t F, int64_t D, int64_t J, int32_t window, const int32_t* s0_host);

/* ---- composite factors (composite_factor.py:137-342) ------------------------------- */
/* composite_factor_calculation preprocessing (:157-178): Adj[k] = suffix-scaled X[cols[k]]
 * with per-(column, date) numpy linear nanpercentiles.  suffix codes 0 none, 1 _eq,
 * 2 _flx, 3 _long, 4 _short; qlo/qhi: device double[5] percentile fractions per code. */
fmx_status fmx_comp_adj(const double* X, const int32_t* cols_dev, const int32_t* suffix_dev, const double* qlo_dev,
                        const double* qhi_dev, double* Adj, int64_t K, int64_t D, int64_t A, void* stream);
/* prefix-group proxies (:181-190): skipna mean over the columns gcols[goff[g]..goff[g+1]). */
fmx_status fmx_comp_proxy(const double* Adj, const int32_t* gcols_dev, const int32_t* goff_dev, double* Prox,
                          int64_t G, int64_t D, int64_t A, void* stream);
/* combine normalised proxies (mode 0 skipna mean / 1 skipna sum) and demean (:204-216). */
fmx_status fmx_comp_combine(const double* Nrm, int64_t G, int64_t D, int64_t A, int32_t mode,
                            const uint8_t* present, double* Out, void* stream);
/* weighted_composite_factor (:220-342): pooled suffix percentiles per selection row j
 * (columns scol[soff[4j+s-1] .. soff[4j+s]) for suffix s=1..4); lohi[J][4][3] = lo, hi, n. */
fmx_status fmx_wcomp_pct(const double* X, const int32_t* pdate, const int32_t* soff, const int32_t* scol, int64_t J,
                         int64_t D, int64_t A, const double* qlo_dev, const double* qhi_dev, double* lohi,
                         void* stream);
/* per-row prefix-group proxies Prox[G][J][A] from the row plan (ncol, col, suf, grp). */
fmx_status fmx_wcomp_proxy(const double* X, const int32_t* pdate, const int32_t* ncol, const int32_t* col,
                           const int32_t* suf, const int32_t* grp, int32_t KMAX, int64_t J, int64_t D, int64_t A,
                           const double* lohi, int64_t G, double* Prox, void* stream);
/* weighted sum of normalised proxies (Python sum, NaN propagates), demean, NaN -> 0,
 * written to Out[pdate[j]][:]. */
fmx_status fmx_wcomp_combine(const double* Nrm, const int32_t* pdate, const int32_t* ngrp, const double* gw,
                             int32_t KMAX, int64_t J, int64_t D, int64_t A, const uint8_t* present, double* Out,
                             void* stream);

/* ---- daily trade list (portfolio_simulation.py:96-170, method 'equal') ------------ */
/* Replaces Simulation._daily_trade_list with _calculate_equal_weights (:156-170) and
 * _normalize_legs (:250-262) over one [D][A] signal panel X (present [D][A] or NULL):
 * Wraw = same-day weights (NaN on absent cells), Wout = per-symbol shift(1) of Wraw
 * over present rows (:151-152), counts [D][2] = (long_count, short_count), NaN on dates
 * with no present row.  A <= 16384. */
fmx_status fmx_trade_equal(const double* X, const uint8_t* present, double* Wraw, double* Wout,
                           double* counts, int64_t D, int64_t A, double pct, void* stream);
/* Method 'linear' (portfolio_simulation.py:172-181): the signal on its positive / negative
 * cells, _normalize_legs (:250-262) and _cap_and_redistribute(max_weight, 10, 1e-6)
 * (:264-313), every pandas sum a numpy pairwise sum over its subset in symbol order
 * (bit-identical); counts = (len(pos), len(neg)).  Same layout as fmx_trade_equal. */
fmx_status fmx_trade_linear(const double* X, const uint8_t* present, double* Wraw, double* Wout,
                            double* counts, int64_t D, int64_t A, double max_weight, void* stream);
/* F trade books in one launch (multi_manager.py:41-49: one manager per factor): X, Wraw,
 * Wout [F][D][A], counts [F][D][2]; method 0 = equal (pct), 1 = linear (max_weight);
 * present [D][A] shared (or NULL); nan_absent = 1 treats NaN cells as no row
 * (factors_df[fac].dropna()). */
fmx_status fmx_trade_books(int32_t method, const double* X, const uint8_t* present, int32_t nan_absent,
                           double* Wraw, double* Wout, double* counts, int64_t F, int64_t D, int64_t A,
                           double pct, double max_weight, void* stream);
/* Per-symbol shift(1) over the present rows of F same-day books W [F][D][A] (present
 * cells are never NaN in a book, absent ones always are): out[f][d][a] = the book's value
 * on the symbol's previous present row (portfolio_simulation.py:151-152). */
fmx_status fmx_shift_rows(const double* W, double* out, int64_t F, int64_t D, int64_t A, void* stream);
/* Replaces multi_manager.compute_multimanager_weights' combination loop (:51-72): Wf
 * [F][D][A] shifted manager books and counts [F][D][2] (NaN on dates a manager has no
 * rows) from fmx_trade_equal; fw [Dw][Fw] factor weights, colmap [Fw] column -> manager
 * (-1: no such factor), wdate [Dw] -> date index.  out [Dw][A], out_counts [Dw][2]. */
fmx_status fmx_mm_combine(const double* Wf, const double* counts, const double* fw, const int32_t* colmap,
                          const int32_t* wdate, double* out, double* out_counts, int64_t Fw, int64_t Dw,
                          int64_t D, int64_t A, void* stream);

/* ---- portfolio P&L (portfolio_simulation.py:748-819) ---------- */
/* Replaces Simulation._daily_portfolio_returns' per-date sums on the aligned [D][A] grid
 * (union of the weights' and returns' dates/symbols; NaN cells count as 0 as after
 * unstack().fillna(0)): W shifted weights, R returns, CAP cap flags (or NULL: no cost),
 * wprev [D] = row of the previous weights date (-1: none).  out [D][6] = (sum longs*r,
 * sum shorts*r, long turnover, short turnover, long cost, short cost); contrib [A][2]
 * (optional) = per-symbol long / short P&L net of cost (contributor=True, :790-793). */
fmx_status fmx_pnl_daily(const double* W, const double* R, const double* CAP, const int32_t* wprev, double* out,
                         double* contrib, int64_t D, int64_t A, void* stream);
/* Replaces _calculate_metrics' daily IC (:799-805): per date, Series.corr (np.corrcoef) of
 * the pair-valid (X, R) cells.  out [D][2] = (n, corr); corr NaN for n < 2 or constant. */
fmx_status fmx_daily_corr(const double* X, const double* R, double* out, int64_t D, int64_t A, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FMX_H_ */
