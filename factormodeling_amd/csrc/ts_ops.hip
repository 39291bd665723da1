// Time-series (per-symbol rolling) kernels.
//
// Reference: operations.py:6-51 (ts_sum/mean/std/zscore/rank/diff/delay/decay/backfill),
// operations.py:185-246 (ts_regression_fast rolling moments) and the builder-defined
// ts_corr (pandas Rolling.corr semantics).  The reference runs
// ``series.groupby(level='symbol').transform(lambda x: x.rolling(w).<agg>())``: a
// sequential walk over each symbol's rows.  Here one lane owns one (factor, asset)
// column of the [F][D][ld] panel and walks its dates; at each date the 64 lanes of a
// wave read 64 consecutive assets (coalesced 512-B rows).
//
// No kernel keeps the window in LDS, so no window length is refused.  The moment and
// shift ops only need the value LEAVING the window: a register ring for the hot windows
// (k_ts_reg, k_ts_set), a re-read of x[d - W] on dense panels (k_ts_rl) or a trailing row
// pointer on ragged ones (k_ts_ptr).  ts_rank / ts_decay need the whole window: k_ts_win
// streams it per tile of dates.  Rows whose presence byte is 0 are not part of the
// symbol's row sequence (the reference's row-based windows on ragged panels).
//
// The add/remove state machines replicate pandas 2.3.3 _libs/window/aggregations.pyx
// (roll_sum / roll_mean / roll_var incl. Kahan compensation, the consecutive-same-
// value guard and zsqrt), so with -ffp-contract=off the outputs are bit-identical to
// pandas.
#include <cstdlib>

#include "fmx_common.hpp"

namespace fmx {

struct SumSt {
  double s, ca, cr, prev;
  int n, same;                 // counts fit 32 bits (n <= D)
  __device__ void init(double first) { s = ca = cr = 0.0; n = 0; same = 0; prev = first; }
  __device__ void add(double v) {
    if (v == v) {
      n += 1;
      double y = v - ca, t = s + y;
      ca = t - s - y; s = t;
      if (v == prev) same += 1; else same = 1;
      prev = v;
    }
  }
  __device__ void remove(double v) {
    if (v == v) {
      n -= 1;
      double y = -v - cr, t = s + y;
      cr = t - s - y; s = t;
    }
  }
  __device__ double result(int64_t minp) const {
    if (n == 0 && minp == 0) return 0.0;
    if (n >= minp) return (same >= n) ? prev * (double)n : s;
    return qnan();
  }
};

struct MeanSt {
  double s, ca, cr, prev;
  int n, neg, same;
  __device__ void init(double first) { s = ca = cr = 0.0; n = neg = same = 0; prev = first; }
  __device__ void add(double v) {
    if (v == v) {
      n += 1;
      double y = v - ca, t = s + y;
      ca = t - s - y; s = t;
      if (__builtin_signbit(v)) neg += 1;
      if (v == prev) same += 1; else same = 1;
      prev = v;
    }
  }
  __device__ void remove(double v) {
    if (v == v) {
      n -= 1;
      double y = -v - cr, t = s + y;
      cr = t - s - y; s = t;
      if (__builtin_signbit(v)) neg -= 1;
    }
  }
  // result() with the division by the count through mdiv (rt[k] = RN(1 / k), k <= window)
  template <class RT>
  __device__ double result_r(int64_t minp, RT rt) const {
    if (n >= minp && n > 0) {
      double r = mdiv(s, (double)n, rt[n]);
      if (same >= n) r = prev;
      else if (neg == 0 && r < 0) r = 0.0;
      else if (neg == n && r > 0) r = 0.0;
      return r;
    }
    return qnan();
  }
  __device__ double result(int64_t minp) const {
    if (n >= minp && n > 0) {
      double r = s / (double)n;
      if (same >= n) r = prev;
      else if (neg == 0 && r < 0) r = 0.0;
      else if (neg == n && r > 0) r = 0.0;
      return r;
    }
    return qnan();
  }
};

struct VarSt {
  double mean, ssq, n, ca, cr, prev;
  int same;
  __device__ void init(double first) { mean = ssq = n = ca = cr = 0.0; same = 0; prev = first; }
  __device__ void add(double v) {
    if (v != v) return;
    n += 1.0;
    if (v == prev) same += 1; else same = 1;
    prev = v;
    double pm = mean - ca;
    double y = v - ca;
    double t = y - mean;
    ca = t + mean - y;
    if (n != 0.0) mean = mean + t / n; else mean = 0.0;
    ssq = ssq + (v - pm) * (v - mean);
  }
  __device__ void remove(double v) {
    if (v == v) {
      n -= 1.0;
      if (n != 0.0) {
        double pm = mean - cr;
        double y = v - cr;
        double t = y - mean;
        cr = t + mean - y;
        mean = mean - t / n;
        ssq = ssq - (v - pm) * (v - mean);
      } else {
        mean = 0.0;
        ssq = 0.0;
      }
    }
  }
  // add / remove / var with every division by a count through mdiv (rt[k] = RN(1 / k))
  template <class RT>
  __device__ void add_r(double v, RT rt) {
    if (v != v) return;
    n += 1.0;
    if (v == prev) same += 1; else same = 1;
    prev = v;
    double pm = mean - ca;
    double y = v - ca;
    double t = y - mean;
    ca = t + mean - y;
    mean = mean + mdiv(t, n, rt[(int)n]);
    ssq = ssq + (v - pm) * (v - mean);
  }
  template <class RT>
  __device__ void remove_r(double v, RT rt) {
    if (v == v) {
      n -= 1.0;
      if (n != 0.0) {
        double pm = mean - cr;
        double y = v - cr;
        double t = y - mean;
        cr = t + mean - y;
        mean = mean - mdiv(t, n, rt[(int)n]);
        ssq = ssq - (v - pm) * (v - mean);
      } else {
        mean = 0.0;
        ssq = 0.0;
      }
    }
  }
  template <class RT>
  __device__ double var_r(int64_t minp, int ddof, RT rt) const {
    if (minp < 1) minp = 1;
    if (n >= (double)minp && n > (double)ddof) {
      if (n == 1.0 || (double)same >= n) return 0.0;
      return mdiv(ssq, n - (double)ddof, rt[(int)n - ddof]);
    }
    return qnan();
  }
  __device__ double var(int64_t minp, int ddof) const {
    if (minp < 1) minp = 1;
    if (n >= (double)minp && n > (double)ddof) {
      if (n == 1.0 || (double)same >= n) return 0.0;
      return ssq / (n - (double)ddof);
    }
    return qnan();
  }
};

// One side (x or y) of ts_corr: a MeanSt and a VarSt fed the same values, sharing what the
// two machines track identically -- the NaN test, the count, the run of equal values and
// its value -- so each add / remove does that bookkeeping once.  Every arithmetic step is
// the two machines' own, in their order (bit-identical results).
struct MVSt {
  double s, cam, crm;          // MeanSt: Kahan sum and its add / remove compensations
  double mean, ssq, cav, crv;  // VarSt: Welford mean, sum of squares, compensations
  double prev;
  int n, neg, same;
  __device__ void init(double first) {
    s = cam = crm = mean = ssq = cav = crv = 0.0;
    n = neg = same = 0;
    prev = first;
  }
  template <class RT>
  __device__ void add_r(double v, RT rt) {
    if (v == v) {
      n += 1;
      const double y = v - cam, t = s + y;
      cam = t - s - y; s = t;
      if (__builtin_signbit(v)) neg += 1;
      if (v == prev) same += 1; else same = 1;
      prev = v;
      const double pm = mean - cav;
      const double y2 = v - cav;
      const double t2 = y2 - mean;
      cav = t2 + mean - y2;
      mean = mean + mdiv(t2, (double)n, rt[n]);
      ssq = ssq + (v - pm) * (v - mean);
    }
  }
  template <class RT>
  __device__ void remove_r(double v, RT rt) {
    if (v == v) {
      n -= 1;
      const double y = -v - crm, t = s + y;
      crm = t - s - y; s = t;
      if (__builtin_signbit(v)) neg -= 1;
      if (n != 0) {
        const double pm = mean - crv;
        const double y2 = v - crv;
        const double t2 = y2 - mean;
        crv = t2 + mean - y2;
        mean = mean - mdiv(t2, (double)n, rt[n]);
        ssq = ssq - (v - pm) * (v - mean);
      } else {
        mean = 0.0;
        ssq = 0.0;
      }
    }
  }
  template <class RT>
  __device__ double mean_r(int64_t minp, RT rt) const {   // MeanSt::result_r
    if (n >= minp && n > 0) {
      double r = mdiv(s, (double)n, rt[n]);
      if (same >= n) r = prev;
      else if (neg == 0 && r < 0) r = 0.0;
      else if (neg == n && r > 0) r = 0.0;
      return r;
    }
    return qnan();
  }
  template <class RT>
  __device__ double var_r(int64_t minp, int ddof, RT rt) const {   // VarSt::var_r
    if (minp < 1) minp = 1;
    if (n >= minp && n > ddof) {
      if (n == 1 || same >= n) return 0.0;
      return mdiv(ssq, (double)(n - ddof), rt[n - ddof]);
    }
    return qnan();
  }
};

__device__ __forceinline__ double zsqrt(double v) { return v < 0 ? 0.0 : sqrt(v); }

// ts_decay's weighted window sum sum_k k x_k (k = 1..W oldest -> newest).  The reference is
// np.dot, i.e. BLAS ddot, whose summation order is the library's (OpenBLAS splits it over
// SIMD lanes): decay is pinned to |delta| <= 1e-13 sum k|x| / sum k, not bit for bit.  TS_DECAY_SPLIT
// interleaved fma chains (k mod S) would shorten the dependent chain of the register-ring
// kernels from W to W / S fmas; measured neutral (ts_set 5.14 / 5.18 vs 5.06 / 5.15 ms per
// 504 dates: the rolling set is bound by its column-walk access pattern), so one chain, the
// oldest-to-newest order k_ts_win also uses.  k_ts_set and k_ts_reg share this function, so
// the fused and the single-operator outputs stay bit-identical (tests/test_gpu_fused.py).
#ifndef TS_DECAY_SPLIT
#define TS_DECAY_SPLIT 1
#endif
template <int W>
__device__ __forceinline__ double decay_dot(const double* ring, int q) {
  constexpr int S = TS_DECAY_SPLIT < W ? TS_DECAY_SPLIT : W;
  double a[S];
#pragma unroll
  for (int j = 0; j < S; ++j) a[j] = 0.0;
#pragma unroll
  for (int k = 1; k <= W; ++k) a[(k - 1) % S] = __builtin_fma(ring[(q + k) % W], (double)k, a[(k - 1) % S]);
  if constexpr (S == 1) return a[0];
  else if constexpr (S == 2) return a[0] + a[1];
  else if constexpr (S == 3) return (a[0] + a[1]) + a[2];
  else return (a[0] + a[1]) + (a[2] + a[3]);
}




// ------------------------------------------------------------------------------------
// Per-column walker state.  i counts the column's present rows.
struct ColState {
  SumSt ss;
  MeanSt ms;
  VarSt vs;
  double last;
  int64_t i;
  int nan_in_win;
  bool first;
  __device__ void init() { i = 0; nan_in_win = 0; first = true; last = qnan(); }
};

// One rolling step of a moment / shift op given the value LEAVING the window (`old`, the
// column's present row c.i - W; only read once c.i >= W).  Where that value comes from is
// the caller's business: a register ring (k_ts_reg), a re-read of x[d - W] on dense panels
// (k_ts_rl) or a trailing row pointer on ragged ones (k_ts_ptr) -- none of which bounds W.
// OP in {SUM, MEAN, STD, VAR, ZSCORE, DIFF, DELAY, BACKFILL}.
template <int OP>
__device__ __forceinline__ double ts_moment(ColState& c, double v, double old, int W) {
  if (c.first) { c.ss.init(v); c.ms.init(v); c.vs.init(v); c.first = false; }
  const bool full = c.i >= W;
  double out;
  if (OP == FMX_TS_SUM) {
    if (full) c.ss.remove(old);
    c.ss.add(v);
    out = c.ss.result(W);
  } else if (OP == FMX_TS_MEAN) {
    if (full) c.ms.remove(old);
    c.ms.add(v);
    out = c.ms.result(W);
  } else if (OP == FMX_TS_STD || OP == FMX_TS_VAR) {
    if (full) c.vs.remove(old);
    c.vs.add(v);
    const double var = c.vs.var(W, 1);
    out = (OP == FMX_TS_VAR) ? var : zsqrt(var);
  } else if (OP == FMX_TS_ZSCORE) {
    if (full) { c.ms.remove(old); c.vs.remove(old); }
    c.ms.add(v); c.vs.add(v);
    const double m = c.ms.result(W);
    double sd = zsqrt(c.vs.var(W, 1));
    if (sd == 0.0) sd = qnan();
    out = (v - m) / sd;
  } else if (OP == FMX_TS_DIFF) {
    out = full ? v - old : qnan();
  } else if (OP == FMX_TS_DELAY) {
    out = full ? old : qnan();
  } else {  // BACKFILL
    if (v == v) c.last = v;
    out = c.last;
  }
  c.i += 1;
  return out;
}

// One rolling step with the window ring in registers: slot q is a compile-time index (the
// caller unrolls its date loop by W), so ring[] stays in VGPRs.  Same state machines and
// operation order as ts_step.
template <int OP, int W>
__device__ __forceinline__ double ts_step_reg(ColState& c, double v, double* ring, int q) {
  if (c.first) { c.ss.init(v); c.ms.init(v); c.vs.init(v); c.first = false; }
  double old = qnan();
  if (OP != FMX_TS_BACKFILL) {
    if (c.i >= W) old = ring[q];
    ring[q] = v;
  }
  double out;
  if (OP == FMX_TS_SUM) {
    if (c.i >= W) c.ss.remove(old);
    c.ss.add(v);
    out = c.ss.result(W);
  } else if (OP == FMX_TS_MEAN) {
    if (c.i >= W) c.ms.remove(old);
    c.ms.add(v);
    out = c.ms.result(W);
  } else if (OP == FMX_TS_STD || OP == FMX_TS_VAR) {
    if (c.i >= W) c.vs.remove(old);
    c.vs.add(v);
    const double var = c.vs.var(W, 1);
    out = (OP == FMX_TS_VAR) ? var : zsqrt(var);
  } else if (OP == FMX_TS_ZSCORE) {
    if (c.i >= W) { c.ms.remove(old); c.vs.remove(old); }
    c.ms.add(v); c.vs.add(v);
    const double m = c.ms.result(W);
    double sd = zsqrt(c.vs.var(W, 1));
    if (sd == 0.0) sd = qnan();
    out = (v - m) / sd;
  } else if (OP == FMX_TS_RANK || OP == FMX_TS_DECAY) {
    if (c.i >= W && old != old) c.nan_in_win -= 1;
    if (v != v) c.nan_in_win += 1;
    if (c.i + 1 < W || c.nan_in_win > 0) {
      out = qnan();
    } else if (OP == FMX_TS_RANK) {
      int less = 0, eq = 0;
#pragma unroll
      for (int k = 0; k < W; ++k) {
        less += (ring[k] < v);
        eq += (ring[k] == v);
      }
      constexpr double RW = 1.0 / (double)W;             // constant divisor: mdiv (bit-identical)
      out = mdiv((double)less + (double)(eq + 1) / 2.0, (double)W, RW);
    } else {
      // oldest element sits in slot q+1 (mod W); weights 1..W oldest->newest
      const double acc = decay_dot<W>(ring, q);
      constexpr double DEN = (double)W * (double)(W + 1) / 2.0, RDEN = 1.0 / DEN;
      out = mdiv(acc, DEN, RDEN);
    }
  } else if (OP == FMX_TS_DIFF) {
    out = (c.i >= W) ? v - old : qnan();
  } else if (OP == FMX_TS_DELAY) {
    out = (c.i >= W) ? old : qnan();
  } else {  // BACKFILL
    if (v == v) c.last = v;
    out = c.last;
  }
  c.i += 1;
  return out;
}

// Dense panels (no presence mask), W in the instantiated set: one lane per (factor,
// asset) column, 256 columns per block; the date loop is unrolled by W so that the ring
// slot of each unrolled step is static, and loads run PF dates ahead (PF divides W).
// Without an LDS ring, occupancy is set by registers alone.
template <int OP, int W, int PF>
__global__ void __launch_bounds__(256, (OP == FMX_TS_SUM || OP == FMX_TS_ZSCORE) ? 4 : 5)
k_ts_reg(const double* __restrict__ X, double* __restrict__ Y, int64_t F, int64_t D, int64_t A, int64_t ld) {
  static_assert(W % PF == 0, "PF must divide W");
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col >= F * A) return;
  const int64_t f = col / A, a = col - f * A;
  const double* x = X + f * D * ld + a;
  double* y = Y + f * D * ld + a;
  ColState c;
  c.init();
  double ring[W];
#pragma unroll
  for (int q = 0; q < W; ++q) ring[q] = 0.0;
  double pf[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) pf[q] = q < D ? x[q * ld] : 0.0;
  const double* xp = x + PF * ld;     // next date to fetch
  double* yp = y;                     // next date to store
  int64_t d0 = 0;
  // full blocks of W dates whose prefetches stay in range: no bounds checks
  for (; d0 + W + PF <= D; d0 += W) {
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const double v = pf[q % PF];
      pf[q % PF] = *xp;
      xp += ld;
      *yp = ts_step_reg<OP, W>(c, v, ring, q);
      yp += ld;
    }
  }
  for (; d0 < D; d0 += W) {
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const int64_t d = d0 + q;
      if (d < D) {
        const double v = pf[q % PF];
        if (d + PF < D) pf[q % PF] = *xp;
        xp += ld;
        *yp = ts_step_reg<OP, W>(c, v, ring, q);
        yp += ld;
      }
    }
  }
}

// Fused rolling set over ONE read of the panel: ts_mean(W), ts_std(W), ts_zscore(W),
// ts_rank(WR) and ts_decay(W) with WR <= W (operations.py:10-48) -- the C2 operator set.
// One lane per (factor, asset) column as k_ts_reg; the W-slot register ring serves all
// five, and the mean / Welford machines are shared, exactly as the separate kernels run
// them (ts_zscore is (v - ts_mean) / ts_std with 0 -> NaN, operations.py:18-21), so each
// output is bit-identical to its single-op kernel.  The rank window is the newest WR
// slots of the same ring.  A null output pointer skips that store.
// Algorithmic bytes: 8 B read + 8 B per requested output per factor·asset·day (48 B for
// all five, vs 80 B for five single-op passes).
#ifndef TS_SET_WAVES
#define TS_SET_WAVES 4
#endif
// TS_SET_MV (default): the set's mean and std machines as one MVSt pair (shared NaN test,
// count and equal-run bookkeeping) with every count division through mdiv on an LDS table
// of RN(1 / k); 0: separate MeanSt / VarSt with IEEE divides (A/B).  Bit-identical.
#ifndef TS_SET_MV
#define TS_SET_MV 1
#endif
struct SetSt {
#if TS_SET_MV
  MVSt mv;
#else
  MeanSt ms;
  VarSt vs;
#endif
  int64_t i;
  int nan_w, nan_r;
  bool first;
};

template <int W, int WR>
__device__ __forceinline__ void ts_set_step(SetSt& c, double v, double* ring, int q, int64_t off,
                                            double* __restrict__ Ym, double* __restrict__ Ys,
                                            double* __restrict__ Yz, double* __restrict__ Yr,
                                            double* __restrict__ Yd, const double* rt) {
  const bool full = c.i >= W;
  const double old = full ? ring[q] : qnan();
  // element leaving the rank window (still in the ring when WR < W)
  const double oldr = (WR == W) ? old : ((c.i >= WR) ? ring[(q + W - WR) % W] : qnan());
  ring[q] = v;
#if TS_SET_MV
  if (c.first) { c.mv.init(v); c.first = false; }
  if (full) c.mv.remove_r(old, rt);
  c.mv.add_r(v, rt);
  const double m = c.mv.mean_r(W, rt);
  const double sd = zsqrt(c.mv.var_r(W, 1, rt));
#else
  (void)rt;
  if (c.first) { c.ms.init(v); c.vs.init(v); c.first = false; }
  if (full) { c.ms.remove(old); c.vs.remove(old); }
  c.ms.add(v); c.vs.add(v);
  const double m = c.ms.result(W);
  const double sd = zsqrt(c.vs.var(W, 1));
#endif
  // outputs are written once and not re-read by this kernel: nontemporal (streaming)
  // stores, +11 % on this 1-read / 5-write column walk (tools/colwalk.hip)
  if (Ym) __builtin_nontemporal_store(m, Ym + off);
  if (Ys) __builtin_nontemporal_store(sd, Ys + off);
  if (Yz) __builtin_nontemporal_store((v - m) / (sd == 0.0 ? qnan() : sd), Yz + off);
  if (full && old != old) c.nan_w -= 1;
  if (c.i >= WR && oldr != oldr) c.nan_r -= 1;
  if (v != v) { c.nan_w += 1; c.nan_r += 1; }
  if (Yr) {
    double o = qnan();
    if (c.i + 1 >= WR && c.nan_r == 0) {
      int less = 0, eq = 0;
#pragma unroll
      for (int k = 0; k < WR; ++k) {
        const double w = ring[(q + W - k) % W];
        less += (w < v);
        eq += (w == v);
      }
      constexpr double RWR = 1.0 / (double)WR;           // constant divisor: mdiv (bit-identical)
      o = mdiv((double)less + (double)(eq + 1) / 2.0, (double)WR, RWR);
    }
    __builtin_nontemporal_store(o, Yr + off);
  }
  if (Yd) {
    double o = qnan();
    if (c.i + 1 >= W && c.nan_w == 0) {
      const double acc = decay_dot<W>(ring, q);
      constexpr double DEN = (double)W * (double)(W + 1) / 2.0, RDEN = 1.0 / DEN;
      o = mdiv(acc, DEN, RDEN);
    }
    __builtin_nontemporal_store(o, Yd + off);
  }
  c.i += 1;
  __builtin_amdgcn_sched_barrier(0);   // keep the unrolled steps' live ranges apart
}

// NT: columns (lanes) per workgroup -- adjacent assets, so one date row of a workgroup is
// NT * 8 contiguous bytes per stream (FMX_TS_SET_NT=512|1024 for A/B; 256 by default)
template <int W, int WR, int PF, int NT = 256>
__global__ void __launch_bounds__(NT, TS_SET_WAVES)
k_ts_set(const double* __restrict__ X, double* __restrict__ Ym, double* __restrict__ Ys, double* __restrict__ Yz,
         double* __restrict__ Yr, double* __restrict__ Yd, int64_t F, int64_t D, int64_t A, int64_t ld) {
  static_assert(W % PF == 0 && WR >= 1 && WR <= W, "windows");
  __shared__ double rt[W + 1];                // RN(1 / k), k <= W (mdiv)
  for (int k = threadIdx.x; k <= W; k += NT) rt[k] = 1.0 / (double)k;
  __syncthreads();
  const int64_t col = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (col >= F * A) return;
  const int64_t f = col / A, a = col - f * A;
  const int64_t off0 = f * D * ld + a;
  const double* xp = X + off0;
  SetSt c;
  c.i = 0; c.nan_w = 0; c.nan_r = 0; c.first = true;
  double ring[W];
#pragma unroll
  for (int q = 0; q < W; ++q) ring[q] = 0.0;
  double pf[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) pf[q] = q < D ? __builtin_nontemporal_load(xp + q * ld) : 0.0;
  xp += PF * ld;
  int64_t off = off0;
  int64_t d0 = 0;
  for (; d0 + W + PF <= D; d0 += W) {
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const double v = pf[q % PF];
      pf[q % PF] = __builtin_nontemporal_load(xp);
      xp += ld;
      ts_set_step<W, WR>(c, v, ring, q, off, Ym, Ys, Yz, Yr, Yd, rt);
      off += ld;
      asm volatile("" : "+v"(off));   // no per-step address precomputation (spills)
    }
  }
  for (; d0 < D; d0 += W) {
#pragma unroll
    for (int q = 0; q < W; ++q) {
      const int64_t d = d0 + q;
      if (d < D) {
        const double v = pf[q % PF];
        if (d + PF < D) pf[q % PF] = __builtin_nontemporal_load(xp);
        xp += ld;
        ts_set_step<W, WR>(c, v, ring, q, off, Ym, Ys, Yz, Yr, Yd, rt);
        off += ld;
      asm volatile("" : "+v"(off));   // no per-step address precomputation (spills)
      }
    }
  }
}

// Dense panels, windows without a register ring (W not instantiated in k_ts_reg, e.g. the
// C5 window of 60): the moment machines only need the value LEAVING the window, which on
// a dense panel is x[d - W] -- re-read from memory instead of kept in a ring (a 60-deep
// LDS ring would hold one wave per 30 KB of LDS).  One lane per (factor, asset) column,
// PF dates of both streams in flight; same state machines and operation order as
// ts_moment, so the outputs are bit-identical to every other path.
// OP in {SUM, MEAN, STD, VAR, ZSCORE, DIFF, DELAY}.
template <int OP, int PF>
__global__ void __launch_bounds__(256)
k_ts_rl(const double* __restrict__ X, double* __restrict__ Y, int64_t F, int64_t D, int64_t A, int64_t ld, int W) {
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col >= F * A) return;
  const int64_t f = col / A, a = col - f * A;
  const double* x = X + f * D * ld + a;
  double* y = Y + f * D * ld + a;
  ColState c;
  c.init();
  for (int64_t d0 = 0; d0 < D; d0 += PF) {
    double v[PF], o[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t d = d0 + q;
      v[q] = d < D ? x[d * ld] : 0.0;
      o[q] = (d < D && d >= W) ? x[(d - W) * ld] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t d = d0 + q;
      if (d >= D) break;
      y[d * ld] = ts_moment<OP>(c, v[q], o[q], W);
    }
  }
}

// ts_mean / ts_std / ts_zscore of one window from ONE MeanSt + VarSt pair (fmx_ts_set's
// moments for any window, dense or ragged): the machines, their order and every output's
// arithmetic are ts_moment's MEAN / STD / ZSCORE paths, so each output is bit-identical to
// its single-op pass.  Outputs may be NULL.
__device__ __forceinline__ void ts_mom3_step(ColState& c, double v, double old, int W, double* ym, double* ys,
                                             double* yz) {
  if (c.first) { c.ms.init(v); c.vs.init(v); c.first = false; }
  if (c.i >= W) { c.ms.remove(old); c.vs.remove(old); }
  c.ms.add(v); c.vs.add(v);
  const double m = c.ms.result(W);
  const double sd = zsqrt(c.vs.var(W, 1));
  if (ym) __builtin_nontemporal_store(m, ym);
  if (ys) __builtin_nontemporal_store(sd, ys);
  if (yz) __builtin_nontemporal_store((v - m) / (sd == 0.0 ? qnan() : sd), yz);
  c.i += 1;
}

// Dense: the leaving value re-read at d - W (k_ts_rl), PF dates of both streams in flight;
// ragged (present != NULL): the trailing row pointer of k_ts_ptr, absent rows NaN.
template <int PF>
__global__ void __launch_bounds__(256)
k_ts_mom3(const double* __restrict__ X, double* __restrict__ Ym, double* __restrict__ Ys, double* __restrict__ Yz,
          int64_t F, int64_t D, int64_t A, int64_t ld, int W, const uint8_t* __restrict__ present) {
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col >= F * A) return;
  const int64_t f = col / A, a = col - f * A;
  const int64_t base = f * D * ld + a;
  const double* x = X + base;
  double* ym = Ym ? Ym + base : nullptr;
  double* ys = Ys ? Ys + base : nullptr;
  double* yz = Yz ? Yz + base : nullptr;
  ColState c;
  c.init();
  if (!present) {
    for (int64_t d0 = 0; d0 < D; d0 += PF) {
      double v[PF], o[PF];
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const int64_t d = d0 + q;
        v[q] = d < D ? x[d * ld] : 0.0;
        o[q] = (d < D && d >= W) ? x[(d - W) * ld] : 0.0;
      }
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        const int64_t d = d0 + q;
        if (d >= D) break;
        ts_mom3_step(c, v[q], o[q], W, ym ? ym + d * ld : nullptr, ys ? ys + d * ld : nullptr,
                     yz ? yz + d * ld : nullptr);
      }
    }
    return;
  }
  const uint8_t* pres = present + a;
  int64_t tail = -1;
  double oldv = 0.0;
  for (int64_t d = 0; d < D; ++d) {
    const double v = x[d * ld];
    if (pres[d * ld] == 0) {
      if (ym) ym[d * ld] = qnan();
      if (ys) ys[d * ld] = qnan();
      if (yz) yz[d * ld] = qnan();
      continue;
    }
    if (tail < 0) { tail = d; oldv = v; }
    double old = 0.0;
    if (c.i >= W) {
      old = oldv;
      do { ++tail; } while (pres[tail * ld] == 0);
      oldv = x[tail * ld];
    }
    ts_mom3_step(c, v, old, W, ym ? ym + d * ld : nullptr, ys ? ys + d * ld : nullptr, yz ? yz + d * ld : nullptr);
  }
}

// Ragged panels (a presence byte per (date, asset); absent rows are not part of the
// symbol's row sequence, operations.py's groupby('symbol') walk): the same column walk,
// with the value leaving the window found by a TRAILING ROW POINTER -- the date of the
// column's present row c.i - W, advanced past absent rows as the window slides.  The
// pointer only moves forward, so a column costs O(D) whatever W is (no ring, no LDS, no
// window cap).  The next leaving value is loaded as soon as the pointer moves, a step
// ahead of its use.  Absent rows get NaN.  present == NULL means every row is present.
// OP in {SUM, MEAN, STD, VAR, ZSCORE, DIFF, DELAY, BACKFILL}.
template <int OP, int PF>
__global__ void __launch_bounds__(256)
k_ts_ptr(const double* __restrict__ X, double* __restrict__ Y, int64_t F, int64_t D, int64_t A, int64_t ld, int W,
         const uint8_t* __restrict__ present) {
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col >= F * A) return;
  const int64_t f = col / A, a = col - f * A;
  const double* x = X + f * D * ld + a;
  double* y = Y + f * D * ld + a;
  const uint8_t* pres = present ? present + a : nullptr;
  ColState c;
  c.init();
  int64_t tail = -1;     // date of present row c.i - W (the next row to leave the window)
  double oldv = 0.0;     // x at `tail`
  for (int64_t d0 = 0; d0 < D; d0 += PF) {
    double v[PF];
    bool p[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t d = d0 + q;
      v[q] = d < D ? x[d * ld] : 0.0;
      p[q] = d < D && (pres == nullptr || pres[d * ld] != 0);
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t d = d0 + q;
      if (d >= D) break;
      if (!p[q]) { y[d * ld] = qnan(); continue; }
      if (tail < 0) { tail = d; oldv = v[q]; }
      double old = 0.0;
      if (OP != FMX_TS_BACKFILL && c.i >= W) {
        old = oldv;
        // present row c.i - W + 1 is at or before d (row d is present): the walk stops there
        do { ++tail; } while (pres != nullptr && pres[tail * ld] == 0);
        oldv = x[tail * ld];
      }
      y[d * ld] = ts_moment<OP>(c, v[q], old, W);
    }
  }
}

// Negative windows of diff / delay (operations.py:34-38 with periods < 0: a LEAD of K
// present rows, x.diff(-K) = x - x.shift(-K)).  Every row first gets NaN; when present
// row i arrives, present row i - K (at the trailing pointer) is final.  Dense or ragged,
// any K.
template <int OP>
__global__ void __launch_bounds__(256)
k_ts_lead_ptr(const double* __restrict__ X, double* __restrict__ Y, int64_t F, int64_t D, int64_t A, int64_t ld,
              int K, const uint8_t* __restrict__ present) {
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col >= F * A) return;
  const int64_t f = col / A, a = col - f * A;
  const double* x = X + f * D * ld + a;
  double* y = Y + f * D * ld + a;
  const uint8_t* pres = present ? present + a : nullptr;
  int64_t i = 0, tail = -1;
  for (int64_t d = 0; d < D; ++d) {
    y[d * ld] = qnan();
    if (pres != nullptr && pres[d * ld] == 0) continue;
    const double v = x[d * ld];
    if (tail < 0) tail = d;
    if (i >= K) {
      const double ov = x[tail * ld];
      y[tail * ld] = (OP == FMX_TS_DIFF) ? ov - v : v;   // same thread wrote its NaN earlier
      do { ++tail; } while (pres != nullptr && pres[tail * ld] == 0);
    }
    ++i;
  }
}

// ts_rank and ts_decay for ANY window, dense or ragged (operations.py:23-32, :40-48).
// Both need the whole window at every row, so instead of a W-deep ring a thread owns a
// TILE of T consecutive dates of one column and streams the W + T - 1 rows that feed them
// once, oldest first, updating all T outputs per row from registers:
//   decay:  acc_t = fma(x_p, k, acc_t) with weight k = p - q_t + W in 1..W (the same
//           oldest->newest fma chain as the register-ring kernel: bit-identical to it);
//   rank:   s_t += 2*(x_p < v_t) + (x_p == v_t), so #less + (#equal + 1)/2 = (s_t + 1)/2
//           (the same half-integer, divided by W); a NaN in the window sets a flag bit.
// p / q_t index the column's PRESENT rows (a ragged symbol's window is its last W rows):
// the thread first walks back from its tile to the (W-1)th present row before it, then
// forward; the lanes of a wave walk the same dates, so every row load is one coalesced
// 512-B access.  Work O(W + T) per T outputs, registers O(T), LDS none -- no window cap.
// Waves: 64 consecutive assets of one (factor, tile); 4 waves per block.
constexpr int TSW_T = 16;
constexpr int TSW_NANBIT = 0x40000000;

__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}

template <int OP, int T>
__global__ void __launch_bounds__(256)
k_ts_win(const double* __restrict__ X, double* __restrict__ Y, int64_t F, int64_t D, int64_t A, int64_t ld, int W,
         const uint8_t* __restrict__ present, int64_t achunks, int64_t ntiles) {
  static_assert(T <= 30, "tile bit mask");
  const int lane = threadIdx.x & 63;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t ac = wid % achunks, rest = wid / achunks;
  const int64_t tile = rest % ntiles, f = rest / ntiles;
  if (f >= F) return;                                   // wave-uniform
  const int64_t a = ac * 64 + lane;
  const bool ok = a < A;
  const double* x = X + f * D * ld + (ok ? a : A - 1);
  const uint8_t* pres = present ? present + (ok ? a : A - 1) : nullptr;
  const int Di = (int)D;
  const int d0 = (int)tile * T;
  const int d1 = min(Di, d0 + T);
  // the tile's own rows: presence bits and (rank) the values being ranked
  unsigned pm = 0;
  double v[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int d = d0 + t;
    const bool in = d < d1;
    v[t] = (OP == FMX_TS_RANK && in) ? x[(int64_t)d * ld] : 0.0;
    if (in && (pres == nullptr || pres[(int64_t)d * ld] != 0)) pm |= 1u << t;
  }
  // window start s: the (W-1)th present row before d0 (or the column's first row)
  int pre, s;
  if (pres == nullptr) {
    pre = min(W - 1, d0);
    s = d0 - pre;
  } else {
    pre = 0;
    s = d0;
    for (int db = d0 - 1;; db -= 8) {
      const bool need = ok && pre < W - 1 && db >= 0;
      if (__ballot(need) == 0) break;
      uint8_t pb[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) pb[k] = (db - k >= 0) ? pres[(int64_t)(db - k) * ld] : 0;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (need && pre < W - 1 && pb[k]) { ++pre; s = db - k; }
    }
  }
  // q_t - W for each present output (q_t = its present-row index counted from s)
  double qW[T];
  {
    int q = pre;
#pragma unroll
    for (int t = 0; t < T; ++t) { qW[t] = (double)(q - W); q += (pm >> t) & 1u; }
  }
  double acc[T];
  int s2[T];
#pragma unroll
  for (int t = 0; t < T; ++t) { acc[t] = 0.0; s2[t] = 0; }
  const double Wd = (double)W;
  const int smin = wave_min_i(ok ? s : d0);
  double pd = 0.0;                                      // present index of the next row
  for (int db = smin; db < d1; db += 8) {
    double u[8];
    bool pu[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int d = db + k;
      u[k] = d < d1 ? x[(int64_t)d * ld] : 0.0;
      pu[k] = d < d1 && d >= s && (pres == nullptr || pres[(int64_t)d * ld] != 0);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (!pu[k]) continue;
      const double uk = u[k];
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const double kk = pd - qW[t];                   // weight of row p in output t's window
        const bool inw = kk >= 1.0 && kk <= Wd;
        if (OP == FMX_TS_DECAY) {
          acc[t] = inw ? __builtin_fma(uk, kk, acc[t]) : acc[t];
        } else {
          const int inc = uk < v[t] ? 2 : (uk == v[t] ? 1 : 0);
          const int nx = (uk != uk) ? (s2[t] | TSW_NANBIT) : (s2[t] + inc);
          s2[t] = inw ? nx : s2[t];
        }
      }
      pd += 1.0;
    }
  }
  if (!ok) return;
  double* y = Y + f * D * ld + a;
  const double den = (double)W * (double)(W + 1) / 2.0;
  const double rden = 1.0 / den, rw = 1.0 / Wd;         // once per thread: mdiv below
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int d = d0 + t;
    if (d >= d1) break;
    double o = qnan();
    if (((pm >> t) & 1u) && qW[t] >= -1.0) {            // a full window of W present rows
      if (OP == FMX_TS_DECAY) o = mdiv(acc[t], den, rden);   // NaN in the window propagates
      else if (s2[t] < TSW_NANBIT) o = mdiv((double)(s2[t] + 1) / 2.0, Wd, rw);
    }
    y[(int64_t)d * ld] = o;
  }
}

// C5's feature (builder-defined): the rolling-W ts_std of each column feeding
// a sign-aligned, volatility-scaled exposure
//     F = sign(C) * (x / ts_std(x, W))      (ts_std == 0 -> NaN, as ts_zscore's replace(0, NaN))
// where C = ts_corr(x, R, W) was computed for the same rows (np.sign semantics: +-0 -> +0,
// NaN -> NaN).  The same Welford machine and operation order as k_ts_rl<STD>, so the
// std is bit-identical to fmx_ts_op(STD) and F to the numpy restatement.
template <int PF, bool FAST>
__global__ void __launch_bounds__(256)
k_ts_cvf_rl(const double* __restrict__ X, const double* __restrict__ C, double* __restrict__ Y, int64_t F,
            int64_t D, int64_t A, int64_t ld, int W) {
  extern __shared__ double rt[];                  // FAST: [W + 1], rt[k] = RN(1 / k) (mdiv)
  if (FAST) {
    for (int k = threadIdx.x; k <= W; k += 256) rt[k] = 1.0 / (double)k;
    __syncthreads();
  }
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col >= F * A) return;
  const int64_t f = col / A, a = col - f * A;
  const double* x = X + f * D * ld + a;
  const double* cc = C + f * D * ld + a;
  double* y = Y + f * D * ld + a;
  ColState c;
  c.init();
  for (int64_t d0 = 0; d0 < D; d0 += PF) {
    double v[PF], o[PF], cv[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t d = d0 + q;
      v[q] = d < D ? x[d * ld] : 0.0;
      o[q] = (d < D && d >= W) ? x[(d - W) * ld] : 0.0;
      cv[q] = d < D ? __builtin_nontemporal_load(cc + d * ld) : 0.0;
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t d = d0 + q;
      if (d >= D) break;
      const double vv = v[q];
      if (c.first) { c.ss.init(vv); c.ms.init(vv); c.vs.init(vv); c.first = false; }
      double sd;
      if (FAST) {
        if (c.i >= W) c.vs.remove_r(o[q], rt);
        c.vs.add_r(vv, rt);
        sd = zsqrt(c.vs.var_r(W, 1, rt));
      } else {
        if (c.i >= W) c.vs.remove(o[q]);
        c.vs.add(vv);
        sd = zsqrt(c.vs.var(W, 1));
      }
      if (sd == 0.0) sd = qnan();
      const double cq = cv[q];
      const double sg = cq > 0.0 ? 1.0 : (cq < 0.0 ? -1.0 : (cq == 0.0 ? 0.0 : cq));
      __builtin_nontemporal_store(sg * (vv / sd), y + d * ld);
      c.i += 1;
    }
  }
}

// ts_corr on dense panels with the leaving values re-read (k_ts_corr's ring is 2W x 64
// doubles of LDS per wave).  Same operation order as k_ts_corr: bit-identical.
template <int PF>
__global__ void __launch_bounds__(256)
k_ts_corr_rl(const double* __restrict__ X, const double* __restrict__ Ycol, double* __restrict__ Out, int64_t F,
             int64_t D, int64_t A, int64_t ld, int64_t y_fstride, int W) {
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col >= F * A) return;
  const int64_t f = col / A, a = col - f * A;
  const double* x = X + f * D * ld + a;
  const double* yc = Ycol + f * y_fstride + a;
  double* o = Out + f * D * ld + a;
  MeanSt mxy, mx, my;
  VarSt vx, vy;
  int64_t i = 0, cnt = 0;
  bool first = true;
  for (int64_t d0 = 0; d0 < D; d0 += PF) {
    double xr[PF], yr[PF], xo[PF], yo[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t d = d0 + q;
      xr[q] = d < D ? x[d * ld] : 0.0;
      yr[q] = d < D ? yc[d * ld] : 0.0;
      const bool old = d < D && d >= W;
      xo[q] = old ? x[(d - W) * ld] : 0.0;
      yo[q] = old ? yc[(d - W) * ld] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t d = d0 + q;
      if (d >= D) break;
      const double xv = xr[q] + 0.0 * yr[q];
      const double yv = yr[q] + 0.0 * xr[q];
      const double pv = xv * yv;
      if (first) { mxy.init(pv); mx.init(xv); my.init(yv); vx.init(xv); vy.init(yv); first = false; }
      if (i >= W) {
        const double ox = xo[q] + 0.0 * yo[q], oy = yo[q] + 0.0 * xo[q];
        mxy.remove(ox * oy); mx.remove(ox); my.remove(oy); vx.remove(ox); vy.remove(oy);
        cnt -= (ox + oy == ox + oy);
      }
      mxy.add(pv); mx.add(xv); my.add(yv); vx.add(xv); vy.add(yv);
      cnt += (xv + yv == xv + yv);
      const double cc = (double)cnt;
      const double num = (mxy.result(W) - mx.result(W) * my.result(W)) * (cc / (cc - 1.0));
      const double den = sqrt(vx.var(W, 1) * vy.var(W, 1));
      o[d * ld] = num / den;
      i += 1;
    }
  }
}

// ts_corr on dense panels, C5's kernel (builder-defined; pandas Rolling.corr): the same
// machines and operation order as k_ts_corr_rl -- bit-identical -- with
//  * every division by a window count (the three means, the two Welford mean updates per
//    add / remove, the two variances, c / (c - 1)) through mdiv on a per-workgroup LDS table
//    of RN(1 / k), k <= W: 10 of the 11 IEEE divides per element become 3-op corrections;
//  * a workgroup = 4 factors x the SAME 64 assets (wave w: factor 4 g + w), so the four waves
//    read each return row R[d], R[d - W] from the CU's L1 instead of once per factor from L2.
constexpr int TSC_MAXW = 4096;                    // table in LDS up to this window
template <int PF>
__global__ void __launch_bounds__(256)
k_ts_corr_fast(const double* __restrict__ X, const double* __restrict__ Ycol, double* __restrict__ Out, int64_t F,
               int64_t D, int64_t A, int64_t ld, int64_t y_fstride, int W, int64_t nab) {
  extern __shared__ double rt[];                  // [W + 1]: rt[k] = RN(1 / k)
  for (int k = threadIdx.x; k <= W; k += 256) rt[k] = 1.0 / (double)k;
  __syncthreads();
  const int64_t ab = blockIdx.x % nab, fg = blockIdx.x / nab;
  const int64_t f = fg * 4 + (threadIdx.x >> 6), a = ab * 64 + (threadIdx.x & 63);
  if (f >= F || a >= A) return;
  const double* x = X + f * D * ld + a;
  const double* yc = Ycol + f * y_fstride + a;
  double* o = Out + f * D * ld + a;
  MeanSt mxy;
  MVSt sx, sy;
  int64_t i = 0, cnt = 0;
  bool first = true;
  for (int64_t d0 = 0; d0 < D; d0 += PF) {
    double xr[PF], yr[PF], xo[PF], yo[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t d = d0 + q;
      xr[q] = d < D ? x[d * ld] : 0.0;
      yr[q] = d < D ? yc[d * ld] : 0.0;
      const bool old = d < D && d >= W;
      xo[q] = old ? x[(d - W) * ld] : 0.0;
      yo[q] = old ? yc[(d - W) * ld] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t d = d0 + q;
      if (d >= D) break;
      const double xv = xr[q] + 0.0 * yr[q];
      const double yv = yr[q] + 0.0 * xr[q];
      const double pv = xv * yv;
      if (first) { mxy.init(pv); sx.init(xv); sy.init(yv); first = false; }
      if (i >= W) {
        const double ox = xo[q] + 0.0 * yo[q], oy = yo[q] + 0.0 * xo[q];
        mxy.remove(ox * oy); sx.remove_r(ox, rt); sy.remove_r(oy, rt);
        cnt -= (ox + oy == ox + oy);
      }
      mxy.add(pv); sx.add_r(xv, rt); sy.add_r(yv, rt);
      cnt += (xv + yv == xv + yv);
      const double cc = (double)cnt;
      const double ratio = cnt >= 2 ? mdiv(cc, cc - 1.0, rt[cnt - 1]) : cc / (cc - 1.0);
      const double num = (mxy.result_r(W, rt) - sx.mean_r(W, rt) * sy.mean_r(W, rt)) * ratio;
      const double den = sqrt(sx.var_r(W, 1, rt) * sy.var_r(W, 1, rt));
      o[d * ld] = num / den;
      i += 1;
    }
  }
}

// C5's feature in the ts_corr pass (fmx_ts_corr_feature): k_ts_corr_fast's machines and
// layout (bit-identical corr) plus the feature's own ts_std(x, W) machine on the raw x
// (k_ts_cvf_rl's VarSt, same order), so the feature
//     sign(corr) * (x / ts_std(x, W))      (ts_std 0 -> NaN; np.sign of a NaN corr is NaN)
// is written while the corr is in registers: the corr panel is not written and read back,
// and x / x[d - W] are read once for both.  C (optional, WC) also receives the corr.
//
#ifdef CF_DIAG_RT
struct CfDiagRt {
  double r;
  __device__ double operator[](int) const { return r; }
};
#endif
template <int PF, bool WC>
__global__ void __launch_bounds__(256)
k_ts_corr_feat(const double* __restrict__ X, const double* __restrict__ Ycol, double* __restrict__ C,
               double* __restrict__ Out, int64_t F, int64_t D, int64_t A, int64_t ld, int64_t y_fstride, int W,
               int64_t nab) {
  extern __shared__ double rt_lds[];              // [W + 1]: rt[k] = RN(1 / k)
  for (int k = threadIdx.x; k <= W; k += 256) rt_lds[k] = 1.0 / (double)k;
  __syncthreads();
#ifdef CF_DIAG_RT
  const CfDiagRt rt{1.0 / (double)W};             // diagnostic (wrong results): no table reads
#else
  const double* rt = rt_lds;
#endif
  const int64_t ab = blockIdx.x % nab, fg = blockIdx.x / nab;
  const int64_t f = fg * 4 + (threadIdx.x >> 6), a = ab * 64 + (threadIdx.x & 63);
  if (f >= F || a >= A) return;
  const double* x = X + f * D * ld + a;
  const double* yc = Ycol + f * y_fstride + a;
  double* o = Out + f * D * ld + a;
  double* cp = WC ? C + f * D * ld + a : nullptr;
  MeanSt mxy;
  MVSt sx, sy;
  VarSt vs;                                       // ts_std(x, W) of the raw x (the feature's)
  int64_t i = 0, cnt = 0;
  bool first = true;
  // software pipeline: the four loads of date d + PF are issued before date d is computed
  // (a ring of PF dates in registers), so each wave keeps a date's HBM / MALL latency in
  // flight across its own arithmetic instead of waiting at the top of every step
  double nx[PF], ny[PF], nxo[PF], nyo[PF];
  auto fetch = [&](int64_t d, int s) {
    const bool in = d < D, old = in && d >= W;
    nx[s] = in ? x[d * ld] : 0.0;
    ny[s] = in ? yc[d * ld] : 0.0;
#ifdef CF_DIAG_NOOLD
    nxo[s] = nx[s];                               // diagnostic (wrong results): no leaving-row reads
    nyo[s] = ny[s];
    (void)old;
#else
    nxo[s] = old ? x[(d - W) * ld] : 0.0;
    nyo[s] = old ? yc[(d - W) * ld] : 0.0;
#endif
  };
#pragma unroll
  for (int q = 0; q < PF; ++q) fetch(q, q);
  for (int64_t d0 = 0; d0 < D; d0 += PF) {
    double xr[PF], yr[PF], xo[PF], yo[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const int64_t d = d0 + q;
      if (d >= D) break;
      xr[q] = nx[q]; yr[q] = ny[q]; xo[q] = nxo[q]; yo[q] = nyo[q];
      fetch(d + PF, q);
      const double xv = xr[q] + 0.0 * yr[q];
      const double yv = yr[q] + 0.0 * xr[q];
      const double pv = xv * yv;
      if (first) { mxy.init(pv); sx.init(xv); sy.init(yv); vs.init(xr[q]); first = false; }
      if (i >= W) {
        const double ox = xo[q] + 0.0 * yo[q], oy = yo[q] + 0.0 * xo[q];
        mxy.remove(ox * oy); sx.remove_r(ox, rt); sy.remove_r(oy, rt);
        cnt -= (ox + oy == ox + oy);
        vs.remove_r(xo[q], rt);
      }
      mxy.add(pv); sx.add_r(xv, rt); sy.add_r(yv, rt);
      cnt += (xv + yv == xv + yv);
      vs.add_r(xr[q], rt);
      const double cc = (double)cnt;
      const double ratio = cnt >= 2 ? mdiv(cc, cc - 1.0, rt[cnt - 1]) : cc / (cc - 1.0);
      const double num = (mxy.result_r(W, rt) - sx.mean_r(W, rt) * sy.mean_r(W, rt)) * ratio;
      const double pv2 = sx.var_r(W, 1, rt) * sy.var_r(W, 1, rt);
      double sg;
      if constexpr (WC) {
        const double cq = num / sqrt(pv2);
        __builtin_nontemporal_store(cq, cp + d * ld);
        sg = cq > 0.0 ? 1.0 : (cq < 0.0 ? -1.0 : (cq == 0.0 ? 0.0 : cq));
      } else {
        // (a sign-only shortcut that skips the sqrt and divide for ordinary num / p measured
        // neutral, 3.35 vs 3.33 ms per 252 dates: this pass is not bound by those VALU ops)
        const double cq = num / sqrt(pv2);
        sg = cq > 0.0 ? 1.0 : (cq < 0.0 ? -1.0 : (cq == 0.0 ? 0.0 : cq));
      }
      double sd = zsqrt(vs.var_r(W, 1, rt));
      if (sd == 0.0) sd = qnan();
      __builtin_nontemporal_store(sg * (xr[q] / sd), o + d * ld);
      i += 1;
    }
  }
}

// W == 0: diff -> x - x, delay -> x, decay -> x (no window).
__global__ void k_ts_window0(const double* __restrict__ X, double* __restrict__ Y, int64_t n_total,
                             int op, const uint8_t* __restrict__ present, int64_t DA, int64_t ld) {
  (void)ld;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n_total; i += stride) {
    double v = X[i];
    bool p = present ? present[i % DA] : true;
    double o = (op == FMX_TS_DIFF) ? v - v : v;
    Y[i] = p ? o : qnan();
  }
}

// ------------------------------------------------------------------------------------
// ts_corr (builder-defined; pandas Rolling.corr) on ragged panels: prep_binary NaN
// propagation, then roll_mean(x*y), roll_mean(x), roll_mean(y), roll_sum(notna) (minp 0),
// roll_var(x), roll_var(y) and  (mxy - mx*my) * (c/(c-1)) / sqrt(vx*vy).  The leaving
// pair is re-read at the trailing row pointer (k_ts_ptr), so any W; same operation order
// as k_ts_corr_rl: bit-identical on a fully present panel.
__global__ void __launch_bounds__(256)
k_ts_corr_ptr(const double* __restrict__ X, const double* __restrict__ Ycol, double* __restrict__ Out, int64_t F,
              int64_t D, int64_t A, int64_t ld, int64_t y_fstride, int W, const uint8_t* __restrict__ present) {
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (col >= F * A) return;
  const int64_t f = col / A, a = col - f * A;
  const double* x = X + f * D * ld + a;
  const double* yc = Ycol + f * y_fstride + a;
  double* o = Out + f * D * ld + a;
  const uint8_t* pres = present ? present + a : nullptr;
  MeanSt mxy, mx, my;
  VarSt vx, vy;
  int64_t i = 0, cnt = 0, tail = -1;
  bool first = true;
  for (int64_t d = 0; d < D; ++d) {
    if (pres != nullptr && pres[d * ld] == 0) { o[d * ld] = qnan(); continue; }
    const double xr = x[d * ld], yr = yc[d * ld];
    const double xv = xr + 0.0 * yr;
    const double yv = yr + 0.0 * xr;
    const double pv = xv * yv;
    if (first) { mxy.init(pv); mx.init(xv); my.init(yv); vx.init(xv); vy.init(yv); first = false; tail = d; }
    if (i >= W) {
      const double txr = x[tail * ld], tyr = yc[tail * ld];
      const double ox = txr + 0.0 * tyr, oy = tyr + 0.0 * txr;
      mxy.remove(ox * oy); mx.remove(ox); my.remove(oy); vx.remove(ox); vy.remove(oy);
      cnt -= (ox + oy == ox + oy);
      do { ++tail; } while (pres != nullptr && pres[tail * ld] == 0);
    }
    mxy.add(pv); mx.add(xv); my.add(yv); vx.add(xv); vy.add(yv);
    cnt += (xv + yv == xv + yv);
    const double c = (double)cnt;
    const double num = (mxy.result(W) - mx.result(W) * my.result(W)) * (c / (c - 1.0));
    const double den = sqrt(vx.var(W, 1) * vy.var(W, 1));
    o[d * ld] = num / den;
    i += 1;
  }
}

// ts_regression_fast rolling moments over the pair-valid rows of one column
// (operations.py:204-240).  `valid` marks rows that survive the reference's dropna()
// (y and the globally shifted x both non-NaN); output NaN elsewhere.  The leaving pair is
// re-read at the trailing valid-row pointer: any W.
__global__ void __launch_bounds__(256)
k_ts_regression_ptr(const double* __restrict__ Yv, const double* __restrict__ Xv, const uint8_t* __restrict__ valid,
                    double* __restrict__ Out, int64_t D, int64_t A, int64_t ld, int W, int rettype) {
  const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (a >= A) return;
  MeanSt mx, my, mxx, mxy, myy;
  int64_t i = 0, tail = -1;
  bool first = true;
  for (int64_t d = 0; d < D; ++d) {
    const int64_t off = d * ld + a;
    if (!valid[off]) { Out[off] = qnan(); continue; }
    const double xv = Xv[off], yv = Yv[off];
    if (first) { mx.init(xv); my.init(yv); mxx.init(xv * xv); mxy.init(xv * yv); myy.init(yv * yv); first = false; tail = d; }
    if (i >= W) {
      const double ox = Xv[tail * ld + a], oy = Yv[tail * ld + a];
      mx.remove(ox); my.remove(oy); mxx.remove(ox * ox); mxy.remove(ox * oy); myy.remove(oy * oy);
      do { ++tail; } while (valid[tail * ld + a] == 0);
    }
    mx.add(xv); my.add(yv); mxx.add(xv * xv); mxy.add(xv * yv); myy.add(yv * yv);
    const double Mx = mx.result(W), My = my.result(W);
    const double cov = mxy.result(W) - Mx * My;
    const double var_x = mxx.result(W) - Mx * Mx;
    const double beta = cov / var_x;
    const double alpha = My - beta * Mx;
    const double fitted = alpha + beta * xv;
    double r;
    switch (rettype) {
      case 0: r = yv - fitted; break;
      case 1: r = alpha; break;
      case 2: r = beta; break;
      case 3: r = fitted; break;
      default: {
        const double var_y = myy.result(W) - My * My;
        r = (cov * cov) / (var_x * var_y);
      }
    }
    Out[off] = r;
    i += 1;
  }
}

// Register-ring kernel for (op, W), or nullptr when W is not an instantiated window.
template <int W, int PF>
static const void* ts_reg_for(int op) {
  switch (op) {
    case FMX_TS_SUM: return (const void*)k_ts_reg<FMX_TS_SUM, W, PF>;
    case FMX_TS_MEAN: return (const void*)k_ts_reg<FMX_TS_MEAN, W, PF>;
    case FMX_TS_STD: return (const void*)k_ts_reg<FMX_TS_STD, W, PF>;
    case FMX_TS_VAR: return (const void*)k_ts_reg<FMX_TS_VAR, W, PF>;
    case FMX_TS_ZSCORE: return (const void*)k_ts_reg<FMX_TS_ZSCORE, W, PF>;
    case FMX_TS_RANK: return (const void*)k_ts_reg<FMX_TS_RANK, W, PF>;
    case FMX_TS_DECAY: return (const void*)k_ts_reg<FMX_TS_DECAY, W, PF>;
    case FMX_TS_DIFF: return (const void*)k_ts_reg<FMX_TS_DIFF, W, PF>;
    case FMX_TS_DELAY: return (const void*)k_ts_reg<FMX_TS_DELAY, W, PF>;
    default: return nullptr;
  }
}

static const void* ts_reg_kernel(int op, int W) {
  switch (W) {
    case 5: return ts_reg_for<5, 5>(op);
    case 10: return ts_reg_for<10, 10>(op);
    case 20: return ts_reg_for<20, 5>(op);
    default: return nullptr;
  }
}

template <int PF>
static const void* ts_col_for(int op, bool ptr) {
  switch (op) {
    case FMX_TS_SUM: return ptr ? (const void*)k_ts_ptr<FMX_TS_SUM, PF> : (const void*)k_ts_rl<FMX_TS_SUM, PF>;
    case FMX_TS_MEAN: return ptr ? (const void*)k_ts_ptr<FMX_TS_MEAN, PF> : (const void*)k_ts_rl<FMX_TS_MEAN, PF>;
    case FMX_TS_STD: return ptr ? (const void*)k_ts_ptr<FMX_TS_STD, PF> : (const void*)k_ts_rl<FMX_TS_STD, PF>;
    case FMX_TS_VAR: return ptr ? (const void*)k_ts_ptr<FMX_TS_VAR, PF> : (const void*)k_ts_rl<FMX_TS_VAR, PF>;
    case FMX_TS_ZSCORE:
      return ptr ? (const void*)k_ts_ptr<FMX_TS_ZSCORE, PF> : (const void*)k_ts_rl<FMX_TS_ZSCORE, PF>;
    case FMX_TS_DIFF: return ptr ? (const void*)k_ts_ptr<FMX_TS_DIFF, PF> : (const void*)k_ts_rl<FMX_TS_DIFF, PF>;
    case FMX_TS_DELAY: return ptr ? (const void*)k_ts_ptr<FMX_TS_DELAY, PF> : (const void*)k_ts_rl<FMX_TS_DELAY, PF>;
    case FMX_TS_BACKFILL: return (const void*)k_ts_ptr<FMX_TS_BACKFILL, PF>;
    default: return nullptr;
  }
}

// k_ts_win launch: one wave per (factor, tile of TSW_T dates, 64 assets), 4 waves a block.
static fmx_status launch_ts_win(int op, const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                                int W, const uint8_t* present, hipStream_t st) {
  FMX_ARG(D < (int64_t)1 << 30, "too many dates for the windowed kernel");
  int64_t achunks = ceil_div(A, 64), ntiles = ceil_div(D, TSW_T);
  const int64_t waves = F * ntiles * achunks;
  FMX_ARG(ceil_div(waves, 4) < (int64_t)1 << 31, "panel too large for one windowed launch");
  const void* k = op == FMX_TS_RANK ? (const void*)k_ts_win<FMX_TS_RANK, TSW_T>
                                    : (const void*)k_ts_win<FMX_TS_DECAY, TSW_T>;
  void* args[] = {(void*)&X, (void*)&Y, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&W,
                  (void*)&present, (void*)&achunks, (void*)&ntiles};
  FMX_HIP(hipLaunchKernel(k, dim3((unsigned)ceil_div(waves, 4)), dim3(256), args, 0, st));
  return FMX_OK;
}

}  // namespace fmx

using namespace fmx;

// Dispatch (no window cap anywhere):
//   dense, W in {5, 10, 20}          -> k_ts_reg (register ring)
//   rank / decay otherwise           -> k_ts_win (date tiles; dense or ragged)
//   other ops, dense                 -> k_ts_rl  (leaving value re-read at d - W)
//   other ops, ragged; backfill      -> k_ts_ptr (trailing row pointer)
//   diff / delay with W < 0 (a lead) -> k_ts_lead_ptr
extern "C" fmx_status fmx_ts_op(int32_t op, const double* X, double* Y, int64_t F, int64_t D, int64_t A,
                                int64_t ld, int32_t window, const uint8_t* present, void* stream) {
  FMX_ARG(X && Y, "null panel");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A, "bad dims");
  FMX_ARG(op >= FMX_TS_SUM && op <= FMX_TS_BACKFILL, "unknown ts op");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  hipStream_t st = as_stream(stream);
  int W = window;
  if (op == FMX_TS_BACKFILL) W = 1;
  if (op == FMX_TS_DECAY && W < 1) {
    FMX_HIP(hipMemcpyAsync(Y, X, sizeof(double) * F * D * ld, hipMemcpyDeviceToDevice, st));
    if (present) {
      int64_t n = F * D * ld;
      k_ts_window0<<<(int)std::min<int64_t>(ceil_div(n, 256), 8192), 256, 0, st>>>(X, Y, n, FMX_TS_DELAY, present, D * ld, ld);
      FMX_LAUNCH_CHECK("k_ts_window0");
    }
    return FMX_OK;
  }
  if ((op == FMX_TS_DIFF || op == FMX_TS_DELAY) && W == 0) {
    int64_t n = F * D * ld;
    k_ts_window0<<<(int)std::min<int64_t>(ceil_div(n, 256), 8192), 256, 0, st>>>(X, Y, n, op, present, D * ld, ld);
    FMX_LAUNCH_CHECK("k_ts_window0");
    return FMX_OK;
  }
  const dim3 cgrid((unsigned)ceil_div(F * A, 256));
  if ((op == FMX_TS_DIFF || op == FMX_TS_DELAY) && W < 0) {
    FMX_ARG(W > INT32_MIN, "window out of range");
    int K = -W;
    const void* k = op == FMX_TS_DIFF ? (const void*)k_ts_lead_ptr<FMX_TS_DIFF> : (const void*)k_ts_lead_ptr<FMX_TS_DELAY>;
    void* largs[] = {(void*)&X, (void*)&Y, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&K, (void*)&present};
    FMX_HIP(hipLaunchKernel(k, cgrid, dim3(256), largs, 0, st));
    return FMX_OK;
  }
  FMX_ARG(W >= 1, "window must be >= 1");
  if (!present && op != FMX_TS_BACKFILL) {
    const void* kr = ts_reg_kernel(op, W);
    if (kr) {
      void* rargs[] = {(void*)&X, (void*)&Y, (void*)&F, (void*)&D, (void*)&A, (void*)&ld};
      FMX_HIP(hipLaunchKernel(kr, cgrid, dim3(256), rargs, 0, st));
      return FMX_OK;
    }
  }
  if (op == FMX_TS_RANK || op == FMX_TS_DECAY) return launch_ts_win(op, X, Y, F, D, A, ld, W, present, st);
  if (!present && op != FMX_TS_BACKFILL) {
    void* rargs[] = {(void*)&X, (void*)&Y, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&W};
    FMX_HIP(hipLaunchKernel(ts_col_for<8>(op, false), cgrid, dim3(256), rargs, 0, st));
    return FMX_OK;
  }
  void* pargs[] = {(void*)&X, (void*)&Y, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&W, (void*)&present};
  FMX_HIP(hipLaunchKernel(ts_col_for<8>(op, true), cgrid, dim3(256), pargs, 0, st));
  return FMX_OK;
}

extern "C" fmx_status fmx_ts_set(const double* X, double* Ymean, double* Ystd, double* Yzscore, double* Yrank,
                                 double* Ydecay, int64_t F, int64_t D, int64_t A, int64_t ld, int32_t window,
                                 int32_t rank_window, const uint8_t* present, void* stream) {
  FMX_ARG(X, "null panel");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A, "bad dims");
  FMX_ARG(window >= 1 && rank_window >= 1, "windows must be >= 1");
  double* outs[5] = {Ymean, Ystd, Yzscore, Yrank, Ydecay};
  for (int k = 0; k < 5; ++k) FMX_ARG(outs[k] != X, "outputs must not alias X");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  if (!present && window == 20 && rank_window == 10 && getenv("FMX_TS_SET_SPLIT") == nullptr) {
    void* args[] = {(void*)&X, (void*)&Ymean, (void*)&Ystd, (void*)&Yzscore, (void*)&Yrank, (void*)&Ydecay,
                    (void*)&F, (void*)&D, (void*)&A, (void*)&ld};
    static const int nt = [] {
      const char* e = getenv("FMX_TS_SET_NT");
      const int v = e ? atoi(e) : 256;
      return (v == 512 || v == 1024) ? v : 256;
    }();
    const void* k = nt == 1024 ? (const void*)k_ts_set<20, 10, 5, 1024>
                    : nt == 512 ? (const void*)k_ts_set<20, 10, 5, 512> : (const void*)k_ts_set<20, 10, 5, 256>;
    FMX_HIP(hipLaunchKernel(k, dim3((unsigned)ceil_div(F * A, nt)), dim3(nt), args, 0, as_stream(stream)));
    return FMX_OK;
  }
  // other windows / ragged panels: the three moments from one pair of machines (one pass),
  // then ts_rank and ts_decay on their own best kernels (any window); FMX_TS_SET_SPLIT=1:
  // one single-op pass per output (A/B)
  const int32_t ops[5] = {FMX_TS_MEAN, FMX_TS_STD, FMX_TS_ZSCORE, FMX_TS_RANK, FMX_TS_DECAY};
  int k0 = 0;
  if (getenv("FMX_TS_SET_SPLIT") == nullptr && (Ymean || Ystd || Yzscore)) {
    int W = window;
    void* args[] = {(void*)&X, (void*)&Ymean, (void*)&Ystd, (void*)&Yzscore, (void*)&F, (void*)&D, (void*)&A,
                    (void*)&ld, (void*)&W, (void*)&present};
    FMX_HIP(hipLaunchKernel((const void*)k_ts_mom3<4>, dim3((unsigned)ceil_div(F * A, 256)), dim3(256), args, 0,
                            as_stream(stream)));
    k0 = 3;
  }
  for (int k = k0; k < 5; ++k) {
    if (!outs[k]) continue;
    fmx_status e = fmx_ts_op(ops[k], X, outs[k], F, D, A, ld, k == 3 ? rank_window : window, present, stream);
    if (e) return e;
  }
  return FMX_OK;
}

extern "C" fmx_status fmx_ts_corr(const double* X, const double* Ycol, double* Out, int64_t F, int64_t D,
                                  int64_t A, int64_t ld, int64_t y_fstride, int32_t window,
                                  const uint8_t* present, void* stream) {
  FMX_ARG(X && Ycol && Out, "null panel");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A, "bad dims");
  FMX_ARG(window >= 1, "window must be >= 1");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  int W = window;
  const dim3 grid((unsigned)ceil_div(F * A, 256));
  if (!present) {   // dense: leaving values re-read at d - W
    void* rargs[] = {(void*)&X, (void*)&Ycol, (void*)&Out, (void*)&F, (void*)&D, (void*)&A, (void*)&ld,
                     (void*)&y_fstride, (void*)&W};
    static const bool v1 = getenv("FMX_TS_CORR_V1") != nullptr;   // A/B: the round-3 kernel
    if (W <= TSC_MAXW && !v1) {
      int64_t nab = ceil_div(A, 64);
      void* fargs[] = {(void*)&X, (void*)&Ycol, (void*)&Out, (void*)&F, (void*)&D, (void*)&A, (void*)&ld,
                       (void*)&y_fstride, (void*)&W, (void*)&nab};
      FMX_HIP(hipLaunchKernel((const void*)k_ts_corr_fast<2>, dim3((unsigned)(nab * ceil_div(F, 4))), dim3(256),
                              fargs, sizeof(double) * (W + 1), as_stream(stream)));
      return FMX_OK;
    }
    // two dates of the four streams in flight: 116 VGPRs, 4 waves/SIMD (four dates: 154
    // VGPRs, 3 waves, 160 vs 156 ms at C5; eight: 180 ms; forcing 4-5 waves spills)
    const void* kc = (const void*)k_ts_corr_rl<2>;
    FMX_HIP(hipLaunchKernel(kc, grid, dim3(256), rargs, 0, as_stream(stream)));
    return FMX_OK;
  }
  void* args[] = {(void*)&X, (void*)&Ycol, (void*)&Out, (void*)&F, (void*)&D, (void*)&A, (void*)&ld,
                  (void*)&y_fstride, (void*)&W, (void*)&present};
  FMX_HIP(hipLaunchKernel((const void*)k_ts_corr_ptr, grid, dim3(256), args, 0, as_stream(stream)));
  return FMX_OK;
}

extern "C" fmx_status fmx_ts_corr_vol_feature(const double* X, const double* C, double* Y, int64_t F, int64_t D,
                                              int64_t A, int64_t ld, int32_t window, void* stream) {
  FMX_ARG(X && C && Y, "null panel");
  FMX_ARG(Y != X && Y != C, "output must not alias the inputs");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A, "bad dims");
  FMX_ARG(window >= 1, "window must be >= 1");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  int W = window;
  void* args[] = {(void*)&X, (void*)&C, (void*)&Y, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&W};
  static const bool v1 = getenv("FMX_TS_CORR_V1") != nullptr;   // A/B: IEEE divides
  const bool fast = W <= TSC_MAXW && !v1;
  FMX_HIP(hipLaunchKernel(fast ? (const void*)k_ts_cvf_rl<8, true> : (const void*)k_ts_cvf_rl<8, false>,
                          dim3((unsigned)ceil_div(F * A, 256)), dim3(256), args, fast ? sizeof(double) * (W + 1) : 0,
                          as_stream(stream)));
  return FMX_OK;
}

extern "C" fmx_status fmx_ts_corr_feature(const double* X, const double* Ycol, double* C, double* Y, int64_t F,
                                          int64_t D, int64_t A, int64_t ld, int64_t y_fstride, int32_t window,
                                          void* stream) {
  FMX_ARG(X && Ycol && Y, "null panel");
  FMX_ARG(Y != X && Y != Ycol && (!C || (C != X && C != Ycol && C != Y)), "outputs must not alias the inputs");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A, "bad dims");
  FMX_ARG(window >= 1 && window <= TSC_MAXW, "window must be in [1, 4096]");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  int W = window;
  int64_t nab = ceil_div(A, 64);
  void* args[] = {(void*)&X, (void*)&Ycol, (void*)&C, (void*)&Y, (void*)&F, (void*)&D, (void*)&A, (void*)&ld,
                  (void*)&y_fstride, (void*)&W, (void*)&nab};
  // one date in flight: 106 VGPRs, 4 waves/SIMD (two: 130 VGPRs, 3 waves); FMX_CORR_FEAT_PF=2 for A/B
  static const bool pf2 = [] {
    const char* e = getenv("FMX_CORR_FEAT_PF");
    return e && e[0] == '2';
  }();
  const void* k = C ? (pf2 ? (const void*)k_ts_corr_feat<2, true> : (const void*)k_ts_corr_feat<1, true>)
                    : (pf2 ? (const void*)k_ts_corr_feat<2, false> : (const void*)k_ts_corr_feat<1, false>);
  FMX_HIP(hipLaunchKernel(k,
                          dim3((unsigned)(nab * ceil_div(F, 4))), dim3(256), args, sizeof(double) * (W + 1),
                          as_stream(stream)));
  return FMX_OK;
}

extern "C" fmx_status fmx_ts_regression(const double* Yv, const double* Xv, const uint8_t* valid, double* Out,
                                        int64_t D, int64_t A, int64_t ld, int32_t window, int32_t rettype,
                                        void* stream) {
  FMX_ARG(Yv && Xv && valid && Out, "null panel");
  FMX_ARG(D >= 0 && A >= 0 && ld >= A, "bad dims");
  FMX_ARG(window >= 1, "window must be >= 1");
  FMX_ARG(rettype == 0 || rettype == 1 || rettype == 2 || rettype == 3 || rettype == 6, "rettype not implemented");
  if (D == 0 || A == 0) return FMX_OK;
  int W = window;
  int rt = rettype;
  void* args[] = {(void*)&Yv, (void*)&Xv, (void*)&valid, (void*)&Out, (void*)&D, (void*)&A, (void*)&ld,
                  (void*)&W, (void*)&rt};
  FMX_HIP(hipLaunchKernel((const void*)k_ts_regression_ptr, dim3((unsigned)ceil_div(A, 256)), dim3(256), args, 0,
                          as_stream(stream)));
  return FMX_OK;
}
