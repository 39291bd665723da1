// Daily information coefficients, window metrics and ICIR top-k selection.
//
// Reference: factor_selector.py:26-73 (single_factor_metrics), :94-139
// (FactorSelector.prepare_selection) and factor_selection_methods.py:6-26
// (icir_top_selector).
//
// k_ic_daily: one workgroup per (factor, return date t, lag L).  The exposure row
// X[f][t-L] and the return row R[t] are read once; pair-valid members (both non-NaN)
// are sorted in LDS to get scipy.rankdata average ranks, and the workgroup reduces the
// Pearson moments of (f, r) and (rank(f), r) plus the beta f.r / f.f.  This replaces the
// reference's F x D Python loop of two pearsonr calls + one rankdata call per group.
//
// k_ic_window: one lane per (job, factor) summarises the daily series over a date
// window [d0, d1) exactly like factor_selector.py:50-59 (entries with n >= 3; NaN ICs
// dropped; mean, std(ddof=1), t-test of betas, share of positive betas).  The rolling
// selector uses jobs [t-W+1, t) -- the reference's double lag-1 shift means each
// window's metrics are lag-2 ICs over the last W-1 window days.
//
// k_select_icir_top: one workgroup per processed day applies icir_top: order by
// rank_IC_IR descending (NaN last, ties by column position), keep > threshold, take
// top_x largest of the chosen column (ties by that order), equal weights.
#include "rowkit.hpp"

namespace fmx {

constexpr int IC_NT = 256;

struct IcLags { int32_t v[8]; };   // passed by value: no device copy of the host lag list

__global__ void __launch_bounds__(IC_NT)
k_ic_daily(const double* __restrict__ X, const double* __restrict__ R, int64_t F, int64_t D, int64_t A,
           int64_t ld, IcLags lags, int P, double* __restrict__ out) {
  extern __shared__ uint64_t keys[];
  uint16_t* idx = (uint16_t*)(keys + P);
  double* dscr = (double*)(((uintptr_t)(idx + P) + 15) & ~(uintptr_t)15);
  int* iscr = (int*)(dscr + 16);
  const int64_t t = blockIdx.x, f = blockIdx.y;
  const int li = blockIdx.z;
  const int L = lags.v[li];
  double* o_n = out + ((int64_t)(li * 4 + 0) * F + f) * D + t;
  double* o_ic = out + ((int64_t)(li * 4 + 1) * F + f) * D + t;
  double* o_ric = out + ((int64_t)(li * 4 + 2) * F + f) * D + t;
  double* o_b = out + ((int64_t)(li * 4 + 3) * F + f) * D + t;
  const int64_t s = t - L;
  if (s < 0 || s >= D) {
    if (threadIdx.x == 0) { *o_n = 0.0; *o_ic = qnan(); *o_ric = qnan(); *o_b = qnan(); }
    return;
  }
  const double* xf = X + (f * D + s) * ld;
  const double* rr = R + t * ld;
  int nl = 0;
  double sf = 0.0, sr = 0.0, rmin = INFINITY, rmax = -INFINITY;
  for (int i = threadIdx.x; i < P; i += IC_NT) {
    uint64_t k = KEY_SENTINEL;
    if (i < A) {
      double fv = xf[i], rv = rr[i];
      if (fv == fv && rv == rv) {
        k = okey(fv);
        nl += 1;
        sf += fv;
        sr += rv;
        rmin = fmin(rmin, rv);
        rmax = fmax(rmax, rv);
      }
    }
    keys[i] = k;
    idx[i] = (uint16_t)i;
  }
  int n;
  block_exscan<IC_NT>(nl, iscr, &n);
  if (n < 3) {
    if (threadIdx.x == 0) { *o_n = (double)n; *o_ic = qnan(); *o_ric = qnan(); *o_b = qnan(); }
    return;
  }
  sf = block_sum<IC_NT>(sf, dscr);
  sr = block_sum<IC_NT>(sr, dscr);
  rmin = block_min<IC_NT>(rmin, dscr);
  rmax = block_max<IC_NT>(rmax, dscr);
  bitonic_sort<IC_NT>(keys, idx, P);
  const double dn = (double)n;
  const double fm = sf / dn, rm = sr / dn, km = (dn + 1.0) / 2.0;
  double sxy = 0, sxx = 0, syy = 0, kxy = 0, kxx = 0, ff = 0, fr = 0;
  for (int p = threadIdx.x; p < n; p += IC_NT) {
    uint64_t k = keys[p];
    int less = lower_bound_u64(keys, 0, p + 1, k);
    int eq = upper_bound_u64(keys, p, n, k) - less;
    double rk = (double)less + (double)(eq + 1) / 2.0;
    int a = idx[p];
    double fv = okey_inv(k);
    fv = xf[a];  // exact original value (okey folds -0.0)
    double rv = rr[a];
    double dx = fv - fm, dy = rv - rm, dk = rk - km;
    sxy += dx * dy; sxx += dx * dx; syy += dy * dy;
    kxy += dk * dy; kxx += dk * dk;
    ff += fv * fv; fr += fv * rv;
  }
  sxy = block_sum<IC_NT>(sxy, dscr);
  sxx = block_sum<IC_NT>(sxx, dscr);
  syy = block_sum<IC_NT>(syy, dscr);
  kxy = block_sum<IC_NT>(kxy, dscr);
  kxx = block_sum<IC_NT>(kxx, dscr);
  ff = block_sum<IC_NT>(ff, dscr);
  fr = block_sum<IC_NT>(fr, dscr);
  if (threadIdx.x == 0) {
    const bool fconst = keys[0] == keys[n - 1];
    const bool rconst = rmin == rmax;
    double ic = qnan(), ric = qnan();
    if (!fconst && !rconst) {
      ic = sxy / sqrt(sxx * syy);
      ic = fmin(1.0, fmax(-1.0, ic));
      ric = kxy / sqrt(kxx * syy);
      ric = fmin(1.0, fmax(-1.0, ric));
    }
    *o_n = dn;
    *o_ic = ic;
    *o_ric = ric;
    *o_b = ff > 0 ? fr / ff : qnan();
  }
}

// Window summary.  daily: [4][F][D] (n, ic, ric, beta) for one lag.  out: [J][F][8] =
// IC, IC_IR, rank_IC, rank_IC_IR, tstat, n_beta (p-value is finished on the host from
// (tstat, n_beta)), pct_pos, n_days.
__global__ void k_ic_window(const double* __restrict__ daily, int64_t F, int64_t D,
                            const int32_t* __restrict__ d0s, const int32_t* __restrict__ d1s, int64_t J,
                            double* __restrict__ out) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= J * F) return;
  // lanes walk consecutive jobs of one factor: rolling windows start on consecutive dates,
  // so the daily-series reads of a wave are coalesced
  const int64_t f = gid / J, j = gid % J;
  const int d0 = max(0, d0s[j]), d1 = min((int)D, d1s[j]);
  const double* dn = daily + (0 * F + f) * D;
  const double* dic = daily + (1 * F + f) * D;
  const double* dric = daily + (2 * F + f) * D;
  const double* db = daily + (3 * F + f) * D;
  double s_ic = 0, s_ric = 0, s_b = 0;
  int n_ic = 0, n_ric = 0, n_b = 0, n_days = 0, n_pos = 0;
  for (int d = d0; d < d1; ++d) {
    if (dn[d] < 3.0) continue;
    n_days += 1;
    double a = dic[d], b = dric[d], c = db[d];
    if (a == a) { s_ic += a; n_ic += 1; }
    if (b == b) { s_ric += b; n_ric += 1; }
    if (c == c) { s_b += c; n_b += 1; n_pos += (c > 0); }
  }
  const double m_ic = n_ic ? s_ic / n_ic : qnan();
  const double m_ric = n_ric ? s_ric / n_ric : qnan();
  const double m_b = n_b ? s_b / n_b : qnan();
  double v_ic = 0, v_ric = 0, v_b = 0;
  for (int d = d0; d < d1; ++d) {
    if (dn[d] < 3.0) continue;
    double a = dic[d], b = dric[d], c = db[d];
    if (a == a) v_ic += (a - m_ic) * (a - m_ic);
    if (b == b) v_ric += (b - m_ric) * (b - m_ric);
    if (c == c) v_b += (c - m_b) * (c - m_b);
  }
  double* o = out + (j * F + f) * 8;
  o[0] = m_ic;
  o[1] = n_ic > 1 ? m_ic / sqrt(v_ic / (n_ic - 1)) : qnan();
  o[2] = m_ric;
  o[3] = n_ric > 1 ? m_ric / sqrt(v_ric / (n_ric - 1)) : qnan();
  if (n_b > 1) {
    double var = (v_b / n_b) * ((double)n_b / (double)(n_b - 1));
    o[4] = m_b / sqrt(var / n_b);
  } else {
    o[4] = qnan();
  }
  o[5] = (double)n_b;
  o[6] = n_b ? (double)n_pos / (double)n_b : qnan();
  o[7] = (double)n_days;
}

// Long windows with few (job, factor) pairs (the full-sample summary: J = 1, so only F
// lanes would walk ~D days each): one 256-thread block per pair, block-reduced sums; same
// outputs as k_ic_window (summation order differs: tolerance-level, not bit-level).
__global__ void __launch_bounds__(256)
k_ic_window_blk(const double* __restrict__ daily, int64_t F, int64_t D, const int32_t* __restrict__ d0s,
                const int32_t* __restrict__ d1s, int64_t J, double* __restrict__ out) {
  __shared__ double scr[16];
  const int64_t j = blockIdx.x / F, f = blockIdx.x % F;
  const int d0 = max(0, d0s[j]), d1 = min((int)D, d1s[j]);
  const double* dn = daily + (0 * F + f) * D;
  const double* dic = daily + (1 * F + f) * D;
  const double* dric = daily + (2 * F + f) * D;
  const double* db = daily + (3 * F + f) * D;
  double s_ic = 0, s_ric = 0, s_b = 0, n_ic = 0, n_ric = 0, n_b = 0, n_days = 0, n_pos = 0;
  for (int d = d0 + (int)threadIdx.x; d < d1; d += 256) {
    if (dn[d] < 3.0) continue;
    n_days += 1;
    const double a = dic[d], b = dric[d], c = db[d];
    if (a == a) { s_ic += a; n_ic += 1; }
    if (b == b) { s_ric += b; n_ric += 1; }
    if (c == c) { s_b += c; n_b += 1; n_pos += (c > 0); }
  }
  s_ic = block_sum<256>(s_ic, scr); s_ric = block_sum<256>(s_ric, scr); s_b = block_sum<256>(s_b, scr);
  n_ic = block_sum<256>(n_ic, scr); n_ric = block_sum<256>(n_ric, scr); n_b = block_sum<256>(n_b, scr);
  n_days = block_sum<256>(n_days, scr); n_pos = block_sum<256>(n_pos, scr);
  const double m_ic = n_ic > 0 ? s_ic / n_ic : qnan();
  const double m_ric = n_ric > 0 ? s_ric / n_ric : qnan();
  const double m_b = n_b > 0 ? s_b / n_b : qnan();
  double v_ic = 0, v_ric = 0, v_b = 0;
  for (int d = d0 + (int)threadIdx.x; d < d1; d += 256) {
    if (dn[d] < 3.0) continue;
    const double a = dic[d], b = dric[d], c = db[d];
    if (a == a) v_ic += (a - m_ic) * (a - m_ic);
    if (b == b) v_ric += (b - m_ric) * (b - m_ric);
    if (c == c) v_b += (c - m_b) * (c - m_b);
  }
  v_ic = block_sum<256>(v_ic, scr); v_ric = block_sum<256>(v_ric, scr); v_b = block_sum<256>(v_b, scr);
  if (threadIdx.x == 0) {
    double* o = out + (j * F + f) * 8;
    o[0] = m_ic;
    o[1] = n_ic > 1 ? m_ic / sqrt(v_ic / (n_ic - 1)) : qnan();
    o[2] = m_ric;
    o[3] = n_ric > 1 ? m_ric / sqrt(v_ric / (n_ric - 1)) : qnan();
    if (n_b > 1) {
      const double var = (v_b / n_b) * (n_b / (n_b - 1));
      o[4] = m_b / sqrt(var / n_b);
    } else {
      o[4] = qnan();
    }
    o[5] = n_b;
    o[6] = n_b > 0 ? n_pos / n_b : qnan();
    o[7] = n_days;
  }
}

// icir_top over J days.  metrics [J][F][8]; col 1 (IC_IR) or 3 (rank_IC_IR).
// order_out [J][F]: factor index at each sorted position.  w_out [J][F] (factor order).
__global__ void k_select_icir_top(const double* __restrict__ metrics, int64_t J, int64_t F, int col,
                                  double thr, int top_x, int32_t* __restrict__ order_out,
                                  double* __restrict__ w_out) {
  extern __shared__ double sm[];
  double* rir = sm;           // [F] rank_IC_IR
  double* cv = sm + F;        // [F] chosen column
  int* pos = (int*)(cv + F);  // [F]
  int* iscr = pos + F;        // [16]
  const int64_t j = blockIdx.x;
  const double* m = metrics + j * F * 8;
  for (int f = threadIdx.x; f < F; f += blockDim.x) {
    rir[f] = m[f * 8 + 3];
    cv[f] = m[f * 8 + col];
  }
  __syncthreads();
  int nnan = 0;
  for (int f = threadIdx.x; f < F; f += blockDim.x) nnan += rir[f] != rir[f];
  int tot_nan;
  block_exscan<256>(nnan, iscr, &tot_nan);
  const int nvalid = (int)F - tot_nan;
  for (int f = threadIdx.x; f < F; f += blockDim.x) {
    double v = rir[f];
    int p = 0;
    if (v == v) {
      for (int g = 0; g < F; ++g) {
        double u = rir[g];
        p += (u > v) || (u == v && g < f);
      }
    } else {
      p = nvalid;
      for (int g = 0; g < f; ++g) p += rir[g] != rir[g];
    }
    pos[f] = p;
    order_out[j * F + p] = f;
  }
  __syncthreads();
  int nsel_l = 0;
  for (int f = threadIdx.x; f < F; f += blockDim.x) {
    double c = cv[f];
    bool cand = c > thr;
    int r = 0;
    if (cand) {
      for (int g = 0; g < F; ++g) {
        double u = cv[g];
        if (!(u > thr)) continue;
        r += (u > c) || (u == c && pos[g] < pos[f]);
      }
    }
    bool sel = cand && r < top_x;
    nsel_l += sel;
    w_out[j * F + f] = sel ? 1.0 : 0.0;
  }
  int k;
  block_exscan<256>(nsel_l, iscr, &k);
  if (k > 0) {
    const double w = 1.0 / (double)k;
    for (int f = threadIdx.x; f < F; f += blockDim.x)
      if (w_out[j * F + f] != 0.0) w_out[j * F + f] = w;
  }
}

}  // namespace fmx

using namespace fmx;

extern "C" fmx_status fmx_ic_daily(const double* X, const double* R, int64_t F, int64_t D, int64_t A, int64_t ld,
                                   const int32_t* lags, int32_t n_lags, double* out, void* stream) {
  FMX_ARG(X && R && out && lags, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  FMX_ARG(n_lags >= 1 && n_lags <= 8, "n_lags");
  for (int i = 0; i < n_lags; ++i) FMX_ARG(lags[i] >= 0, "lags must be >= 0");
  if (F == 0 || D == 0) return FMX_OK;
  if (A <= 16384) {
    const fmx_status e = br_ic_daily(X, R, F, D, A, ld, lags, n_lags, out, as_stream(stream));
    if (e != FMX_ERR_UNSUPPORTED) return e;
  }
  // very wide rows: one LDS-bitonic workgroup per (factor, date, lag)
  int P = next_pow2((int)std::max<int64_t>(A, 2));
  size_t lds = (size_t)P * 10 + 16 + 16 * 8 + 16 * 4 + 64;
  if (lds > 160 * 1024) {
    set_error("A too large for the IC kernels' LDS (A <= 12288; longer rows: fmx_ic_daily_ranked)");
    return FMX_ERR_UNSUPPORTED;
  }
  IcLags lv{};
  for (int i = 0; i < n_lags; ++i) lv.v[i] = lags[i];
  hipStream_t st = as_stream(stream);
  if (lds > 64 * 1024)
    FMX_HIP(hipFuncSetAttribute((const void*)k_ic_daily, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  k_ic_daily<<<dim3((unsigned)D, (unsigned)F, (unsigned)n_lags), IC_NT, lds, st>>>(X, R, F, D, A, ld, lv, P, out);
  FMX_LAUNCH_CHECK("k_ic_daily");
  return FMX_OK;
}

extern "C" int64_t fmx_ic_ranked_work_len(int64_t F, int64_t D) { return ic_ranked_work_len(F, D); }

extern "C" fmx_status fmx_ic_daily_ranked(const double* X, const fmx_rank2_t* rank2, const double* R, int64_t F,
                                          int64_t D, int64_t A, int64_t ld, const int32_t* lags, int32_t n_lags,
                                          int32_t* work, int64_t work_len, double* out, void* stream) {
  FMX_ARG(X && rank2 && R && out && lags && work, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 16384, "bad dims (A <= 16384)");
  FMX_ARG(n_lags >= 1 && n_lags <= 8, "n_lags");
  FMX_ARG(work_len >= ic_ranked_work_len(F, D), "work shorter than fmx_ic_ranked_work_len(F, D)");
  for (int i = 0; i < n_lags; ++i) FMX_ARG(lags[i] >= 0, "lags must be >= 0");
  if (F == 0 || D == 0) return FMX_OK;
  return br_ic_ranked(X, rank2, R, F, D, A, ld, lags, n_lags, out, work, as_stream(stream));
}

extern "C" int64_t fmx_rank_ic_work_len(int64_t F, int64_t D, int64_t A) { return rank_ic_work_len(F, D, A); }

extern "C" fmx_status fmx_cs_rank_winsor_ic(const double* X, double* Yrank, double* Ywinsor, const double* R,
                                            int64_t F, int64_t D, int64_t A, int64_t ld, double qlo, double qhi,
                                            const int32_t* lags, int32_t n_lags, fmx_rank2_t* rank2, int32_t* work,
                                            int64_t work_len, double* out, void* stream) {
  FMX_ARG(X && R && out && lags && rank2 && work, "null pointer");
  FMX_ARG((Yrank == nullptr) == (Ywinsor == nullptr), "Yrank and Ywinsor: both or neither");
  FMX_ARG(!Yrank || (Yrank != X && Ywinsor != X && Yrank != Ywinsor), "outputs must be distinct from X and each other");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 16384, "bad dims (A <= 16384)");
  FMX_ARG(n_lags >= 1 && n_lags <= 2, "n_lags 1 or 2");
  FMX_ARG(work_len >= rank_ic_work_len(F, D, A), "work shorter than fmx_rank_ic_work_len(F, D, A)");
  for (int i = 0; i < n_lags; ++i) FMX_ARG(lags[i] >= 0, "lags must be >= 0");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  return br_cs_rank_winsor_ic(X, Yrank, Ywinsor, R, F, D, A, ld, qlo, qhi, lags, n_lags, rank2, work, out,
                              as_stream(stream));
}

extern "C" fmx_status fmx_ic_window(const double* daily, int64_t F, int64_t D, const int32_t* d0_dev,
                                    const int32_t* d1_dev, int64_t J, double* out, void* stream) {
  FMX_ARG(daily && d0_dev && d1_dev && out, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && J >= 0, "bad dims");
  if (F == 0 || J == 0) return FMX_OK;
  int64_t n = J * F;
  if (n <= 4096 && D >= 512) {   // few long summaries: a block per (job, factor)
    k_ic_window_blk<<<(unsigned)n, 256, 0, as_stream(stream)>>>(daily, F, D, d0_dev, d1_dev, J, out);
    FMX_LAUNCH_CHECK("k_ic_window_blk");
    return FMX_OK;
  }
  k_ic_window<<<(unsigned)ceil_div(n, 256), 256, 0, as_stream(stream)>>>(daily, F, D, d0_dev, d1_dev, J, out);
  FMX_LAUNCH_CHECK("k_ic_window");
  return FMX_OK;
}

extern "C" fmx_status fmx_select_icir_top(const double* metrics, int64_t J, int64_t F, int32_t use_rank_icir,
                                          double threshold, int32_t top_x, int32_t* order_out, double* w_out,
                                          void* stream) {
  FMX_ARG(metrics && order_out && w_out, "null pointer");
  FMX_ARG(J >= 0 && F >= 0, "bad dims");
  if (J == 0 || F == 0) return FMX_OK;
  size_t lds = (size_t)F * 20 + 16 * 4 + 64;
  FMX_ARG(lds <= 160 * 1024, "too many factors for the selection kernel");
  if (lds > 64 * 1024)
    FMX_HIP(hipFuncSetAttribute((const void*)k_select_icir_top, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int col = use_rank_icir ? 3 : 1;
  int tx = top_x;
  void* args[] = {(void*)&metrics, (void*)&J, (void*)&F, (void*)&col, (void*)&threshold, (void*)&tx,
                  (void*)&order_out, (void*)&w_out};
  FMX_HIP(hipLaunchKernel((const void*)k_select_icir_top, dim3((unsigned)J), dim3(256), args, lds,
                          as_stream(stream)));
  return FMX_OK;
}
