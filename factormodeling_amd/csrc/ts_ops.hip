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
// The window history is a thread-private ring in LDS laid out ring[slot*64 + lane]
// (bank-conflict free, no barriers).  Rows whose presence byte is 0 are skipped: the
// ring only advances on present rows, which reproduces the reference's row-based
// windows on ragged panels.
//
// The add/remove state machines replicate pandas 2.3.3 _libs/window/aggregations.pyx
// (roll_sum / roll_mean / roll_var incl. Kahan compensation, the consecutive-same-
// value guard and zsqrt), so with -ffp-contract=off the outputs are bit-identical to
// pandas.
#include <cstdlib>

#include "fmx_common.hpp"

namespace fmx {

constexpr int TS_BLOCK = 64;   // one wave per block: the LDS ring is thread-private
constexpr int TS_UNROLL = 8;   // dates prefetched per lane

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
  __device__ double var(int64_t minp, int ddof) const {
    if (minp < 1) minp = 1;
    if (n >= (double)minp && n > (double)ddof) {
      if (n == 1.0 || (double)same >= n) return 0.0;
      return ssq / (n - (double)ddof);
    }
    return qnan();
  }
};

__device__ __forceinline__ double zsqrt(double v) { return v < 0 ? 0.0 : sqrt(v); }

// ------------------------------------------------------------------------------------
// Per-column walker state.  i counts the column's present rows; the column's window lives
// in the LDS ring at ring[(slot * TS_BLOCK + lane) * V + u].
struct ColState {
  SumSt ss;
  MeanSt ms;
  VarSt vs;
  double last;
  int64_t i;
  int slot, nan_in_win;
  bool first;
  __device__ void init() { i = 0; slot = 0; nan_in_win = 0; first = true; last = qnan(); }
};

template <int OP, int V>
__device__ __forceinline__ double ts_step(ColState& c, double v, int W, double* ring, int lane, int u) {
  if (c.first) { c.ss.init(v); c.ms.init(v); c.vs.init(v); c.first = false; }
  double old = qnan();
  if (OP != FMX_TS_BACKFILL) {
    double* rs = ring + ((int64_t)c.slot * TS_BLOCK + lane) * V + u;
    if (c.i >= W) old = *rs;
    *rs = v;
    c.slot = (c.slot + 1 == W) ? 0 : c.slot + 1;
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
      for (int k = 0; k < W; ++k) {
        const double w = ring[((int64_t)k * TS_BLOCK + lane) * V + u];
        less += (w < v);
        eq += (w == v);
      }
      out = ((double)less + (double)(eq + 1) / 2.0) / (double)W;
    } else {
      // oldest element sits at `slot` (just advanced); weights 1..W oldest->newest
      double acc = 0.0;
      int sl = c.slot;
      for (int k = 1; k <= W; ++k) {   // fused multiply-adds, as numpy's BLAS ddot
        acc = __builtin_fma(ring[((int64_t)sl * TS_BLOCK + lane) * V + u], (double)k, acc);
        sl = (sl + 1 == W) ? 0 : sl + 1;
      }
      out = acc / ((double)W * (double)(W + 1) / 2.0);
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
      out = ((double)less + (double)(eq + 1) / 2.0) / (double)W;
    } else {
      // oldest element sits in slot q+1 (mod W); weights 1..W oldest->newest
      double acc = 0.0;
#pragma unroll
      for (int k = 1; k <= W; ++k) acc = __builtin_fma(ring[(q + k) % W], (double)k, acc);   // as BLAS ddot
      out = acc / ((double)W * (double)(W + 1) / 2.0);
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
struct SetSt {
  MeanSt ms;
  VarSt vs;
  int64_t i;
  int nan_w, nan_r;
  bool first;
};

template <int W, int WR>
__device__ __forceinline__ void ts_set_step(SetSt& c, double v, double* ring, int q, int64_t off,
                                            double* __restrict__ Ym, double* __restrict__ Ys,
                                            double* __restrict__ Yz, double* __restrict__ Yr,
                                            double* __restrict__ Yd) {
  if (c.first) { c.ms.init(v); c.vs.init(v); c.first = false; }
  const bool full = c.i >= W;
  const double old = full ? ring[q] : qnan();
  // element leaving the rank window (still in the ring when WR < W)
  const double oldr = (WR == W) ? old : ((c.i >= WR) ? ring[(q + W - WR) % W] : qnan());
  ring[q] = v;
  if (full) { c.ms.remove(old); c.vs.remove(old); }
  c.ms.add(v); c.vs.add(v);
  const double m = c.ms.result(W);
  const double sd = zsqrt(c.vs.var(W, 1));
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
      o = ((double)less + (double)(eq + 1) / 2.0) / (double)WR;
    }
    __builtin_nontemporal_store(o, Yr + off);
  }
  if (Yd) {
    double o = qnan();
    if (c.i + 1 >= W && c.nan_w == 0) {
      double acc = 0.0;
#pragma unroll
      for (int k = 1; k <= W; ++k) acc = __builtin_fma(ring[(q + k) % W], (double)k, acc);
      o = acc / ((double)W * (double)(W + 1) / 2.0);
    }
    __builtin_nontemporal_store(o, Yd + off);
  }
  c.i += 1;
  __builtin_amdgcn_sched_barrier(0);   // keep the unrolled steps' live ranges apart
}

template <int W, int WR, int PF>
__global__ void __launch_bounds__(256, TS_SET_WAVES)
k_ts_set(const double* __restrict__ X, double* __restrict__ Ym, double* __restrict__ Ys, double* __restrict__ Yz,
         double* __restrict__ Yr, double* __restrict__ Yd, int64_t F, int64_t D, int64_t A, int64_t ld) {
  static_assert(W % PF == 0 && WR >= 1 && WR <= W, "windows");
  const int64_t col = (int64_t)blockIdx.x * 256 + threadIdx.x;
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
      ts_set_step<W, WR>(c, v, ring, q, off, Ym, Ys, Yz, Yr, Yd);
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
        ts_set_step<W, WR>(c, v, ring, q, off, Ym, Ys, Yz, Yr, Yd);
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
// ts_step, so the outputs are bit-identical.  OP in {SUM, MEAN, STD, VAR, ZSCORE}.
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
      const double vv = v[q];
      if (c.first) { c.ss.init(vv); c.ms.init(vv); c.vs.init(vv); c.first = false; }
      const bool full = c.i >= W;
      double out;
      if (OP == FMX_TS_SUM) {
        if (full) c.ss.remove(o[q]);
        c.ss.add(vv);
        out = c.ss.result(W);
      } else if (OP == FMX_TS_MEAN) {
        if (full) c.ms.remove(o[q]);
        c.ms.add(vv);
        out = c.ms.result(W);
      } else if (OP == FMX_TS_STD || OP == FMX_TS_VAR) {
        if (full) c.vs.remove(o[q]);
        c.vs.add(vv);
        const double var = c.vs.var(W, 1);
        out = (OP == FMX_TS_VAR) ? var : zsqrt(var);
      } else {  // ZSCORE
        if (full) { c.ms.remove(o[q]); c.vs.remove(o[q]); }
        c.ms.add(vv); c.vs.add(vv);
        const double m = c.ms.result(W);
        double sd = zsqrt(c.vs.var(W, 1));
        if (sd == 0.0) sd = qnan();
        out = (vv - m) / sd;
      }
      y[d * ld] = out;
      c.i += 1;
    }
  }
}

// C5's feature (builder-defined): the rolling-W ts_std of each column feeding
// a sign-aligned, volatility-scaled exposure
//     F = sign(C) * (x / ts_std(x, W))      (ts_std == 0 -> NaN, as ts_zscore's replace(0, NaN))
// where C = ts_corr(x, R, W) was computed for the same rows (np.sign semantics: +-0 -> +0,
// NaN -> NaN).  The same Welford machine and operation order as k_ts_rl<STD>, so the
// std is bit-identical to fmx_ts_op(STD) and F to the numpy restatement.
template <int PF>
__global__ void __launch_bounds__(256)
k_ts_cvf_rl(const double* __restrict__ X, const double* __restrict__ C, double* __restrict__ Y, int64_t F,
            int64_t D, int64_t A, int64_t ld, int W) {
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
      if (c.i >= W) c.vs.remove(o[q]);
      c.vs.add(vv);
      double sd = zsqrt(c.vs.var(W, 1));
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

typedef double dbl2 __attribute__((ext_vector_type(2)));

// One lane owns V adjacent assets of one factor (V = 2: 16-byte loads/stores) and walks
// the dates with TS_UNROLL rows of loads in flight.
template <int OP, int V>
__global__ void __launch_bounds__(TS_BLOCK)
k_ts(const double* __restrict__ X, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld,
     int W, const uint8_t* __restrict__ present) {
  extern __shared__ double ring[];  // [W][TS_BLOCK][V]
  const int lane = threadIdx.x;
  const int64_t a = ((int64_t)blockIdx.x * TS_BLOCK + lane) * V;
  if (a >= A) return;
  const int64_t f = blockIdx.y;
  const double* x = X + f * D * ld + a;
  double* y = Y + f * D * ld + a;
  const uint8_t* pres = present ? present + a : nullptr;
  ColState cs[V];
#pragma unroll
  for (int u = 0; u < V; ++u) cs[u].init();
  for (int64_t d0 = 0; d0 < D; d0 += TS_UNROLL) {
    double v[TS_UNROLL][V];
    uint8_t p[TS_UNROLL][V];
#pragma unroll
    for (int q = 0; q < TS_UNROLL; ++q) {
      const int64_t d = d0 + q;
      if (d < D) {
        if (V == 2) {
          const dbl2 t = *reinterpret_cast<const dbl2*>(x + d * ld);
          v[q][0] = t[0];
          v[q][V - 1] = t[1];
        } else {
          v[q][0] = x[d * ld];
        }
#pragma unroll
        for (int u = 0; u < V; ++u) p[q][u] = pres ? pres[d * ld + u] : 1;
      } else {
#pragma unroll
        for (int u = 0; u < V; ++u) p[q][u] = 0;
      }
    }
#pragma unroll
    for (int q = 0; q < TS_UNROLL; ++q) {
      const int64_t d = d0 + q;
      if (d >= D) continue;
      double o[V];
#pragma unroll
      for (int u = 0; u < V; ++u) o[u] = p[q][u] ? ts_step<OP, V>(cs[u], v[q][u], W, ring, lane, u) : qnan();
      if (V == 2) {
        dbl2 t;
        t[0] = o[0];
        t[1] = o[V - 1];
        *reinterpret_cast<dbl2*>(y + d * ld) = t;
      } else {
        y[d * ld] = o[0];
      }
    }
  }
}

// W == 0: diff -> x - x, delay -> x, decay -> x (no ring).
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

// Negative window for diff/delay: a lead by K=-W present rows.  Each row first gets NaN
// and is overwritten once the row K steps ahead arrives.
template <int OP>
__global__ void __launch_bounds__(TS_BLOCK)
k_ts_lead(const double* __restrict__ X, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld,
          int K, const uint8_t* __restrict__ present) {
  extern __shared__ double ring[];  // values [K][64] then positions [K][64]
  double* rpos = ring + (int64_t)K * TS_BLOCK;
  const int lane = threadIdx.x;
  const int64_t a = (int64_t)blockIdx.x * TS_BLOCK + lane;
  if (a >= A) return;
  const int64_t f = blockIdx.y;
  const double* x = X + f * D * ld + a;
  double* y = Y + f * D * ld + a;
  int64_t i = 0;
  int slot = 0;
  for (int64_t d = 0; d < D; ++d) {
    bool p = present ? present[d * ld + a] != 0 : true;
    y[d * ld] = qnan();
    if (!p) continue;
    double v = x[d * ld];
    if (i >= K) {
      double ov = ring[slot * TS_BLOCK + lane];
      int64_t od = (int64_t)rpos[slot * TS_BLOCK + lane];
      y[od * ld] = (OP == FMX_TS_DIFF) ? ov - v : v;
    }
    ring[slot * TS_BLOCK + lane] = v;
    rpos[slot * TS_BLOCK + lane] = (double)d;
    slot = (slot + 1 == K) ? 0 : slot + 1;
    i += 1;
  }
}

// ------------------------------------------------------------------------------------
// ts_corr (builder-defined; pandas Rolling.corr): prep_binary NaN propagation, then
// roll_mean(x*y), roll_mean(x), roll_mean(y), roll_sum(notna) (minp 0), roll_var(x),
// roll_var(y) and  (mxy - mx*my) * (c/(c-1)) / sqrt(vx*vy).
__global__ void __launch_bounds__(TS_BLOCK)
k_ts_corr(const double* __restrict__ X, const double* __restrict__ Ycol, double* __restrict__ Out,
          int64_t D, int64_t A, int64_t ld, int64_t y_fstride, int W,
          const uint8_t* __restrict__ present) {
  extern __shared__ double ring[];  // x [W][64], y [W][64]
  double* ringy = ring + (int64_t)W * TS_BLOCK;
  const int lane = threadIdx.x;
  const int64_t a = (int64_t)blockIdx.x * TS_BLOCK + lane;
  if (a >= A) return;
  const int64_t f = blockIdx.y;
  const double* x = X + f * D * ld + a;
  const double* yc = Ycol + f * y_fstride + a;
  double* o = Out + f * D * ld + a;
  MeanSt mxy, mx, my;
  VarSt vx, vy;
  int64_t i = 0, cnt = 0;
  int slot = 0;
  bool first = true;
  for (int64_t d = 0; d < D; ++d) {
    bool p = present ? present[d * ld + a] != 0 : true;
    if (!p) { o[d * ld] = qnan(); continue; }
    double xr = x[d * ld], yr = yc[d * ld];
    double xv = xr + 0.0 * yr;
    double yv = yr + 0.0 * xr;
    double pv = xv * yv;
    if (first) { mxy.init(pv); mx.init(xv); my.init(yv); vx.init(xv); vy.init(yv); first = false; }
    if (i >= W) {
      double ox = ring[slot * TS_BLOCK + lane], oy = ringy[slot * TS_BLOCK + lane];
      mxy.remove(ox * oy); mx.remove(ox); my.remove(oy); vx.remove(ox); vy.remove(oy);
      cnt -= (ox + oy == ox + oy);
    }
    ring[slot * TS_BLOCK + lane] = xv;
    ringy[slot * TS_BLOCK + lane] = yv;
    slot = (slot + 1 == W) ? 0 : slot + 1;
    mxy.add(pv); mx.add(xv); my.add(yv); vx.add(xv); vy.add(yv);
    cnt += (xv + yv == xv + yv);
    double c = (double)cnt;
    double num = (mxy.result(W) - mx.result(W) * my.result(W)) * (c / (c - 1.0));
    double den = sqrt(vx.var(W, 1) * vy.var(W, 1));
    o[d * ld] = num / den;
    i += 1;
  }
}

// ts_regression_fast rolling moments over the pair-valid rows of one column
// (operations.py:204-240).  `valid` marks rows that survive the reference's dropna()
// (y and the globally shifted x both non-NaN).  Output NaN elsewhere.
__global__ void __launch_bounds__(TS_BLOCK)
k_ts_regression(const double* __restrict__ Yv, const double* __restrict__ Xv,
                const uint8_t* __restrict__ valid, double* __restrict__ Out, int64_t D, int64_t A,
                int64_t ld, int W, int rettype) {
  extern __shared__ double ring[];  // x [W][64], y [W][64]
  double* ringy = ring + (int64_t)W * TS_BLOCK;
  const int lane = threadIdx.x;
  const int64_t a = (int64_t)blockIdx.x * TS_BLOCK + lane;
  if (a >= A) return;
  MeanSt mx, my, mxx, mxy, myy;
  int64_t i = 0;
  int slot = 0;
  bool first = true;
  for (int64_t d = 0; d < D; ++d) {
    int64_t off = d * ld + a;
    if (!valid[off]) { Out[off] = qnan(); continue; }
    double xv = Xv[off], yv = Yv[off];
    if (first) { mx.init(xv); my.init(yv); mxx.init(xv * xv); mxy.init(xv * yv); myy.init(yv * yv); first = false; }
    if (i >= W) {
      double ox = ring[slot * TS_BLOCK + lane], oy = ringy[slot * TS_BLOCK + lane];
      mx.remove(ox); my.remove(oy); mxx.remove(ox * ox); mxy.remove(ox * oy); myy.remove(oy * oy);
    }
    ring[slot * TS_BLOCK + lane] = xv;
    ringy[slot * TS_BLOCK + lane] = yv;
    slot = (slot + 1 == W) ? 0 : slot + 1;
    mx.add(xv); my.add(yv); mxx.add(xv * xv); mxy.add(xv * yv); myy.add(yv * yv);
    double Mx = mx.result(W), My = my.result(W);
    double cov = mxy.result(W) - Mx * My;
    double var_x = mxx.result(W) - Mx * Mx;
    double beta = cov / var_x;
    double alpha = My - beta * Mx;
    double fitted = alpha + beta * xv;
    double r;
    switch (rettype) {
      case 0: r = yv - fitted; break;
      case 1: r = alpha; break;
      case 2: r = beta; break;
      case 3: r = fitted; break;
      default: {
        double var_y = myy.result(W) - My * My;
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

static fmx_status launch_ring(const void* kern, dim3 grid, size_t lds, hipStream_t st, void** args) {
  if (lds > 160 * 1024) {
    set_error("window too large for the LDS ring (needs " + std::to_string(lds) + " bytes)");
    return FMX_ERR_UNSUPPORTED;
  }
  if (lds > 64 * 1024) FMX_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  FMX_HIP(hipLaunchKernel(kern, grid, dim3(TS_BLOCK), args, lds, st));
  return FMX_OK;
}

}  // namespace fmx

using namespace fmx;

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
  // two adjacent assets per lane (16-byte accesses) when rows stay 16-byte aligned
  const bool v2 = (ld % 2 == 0) && (A % 2 == 0) && ((uintptr_t)X % 16 == 0) && ((uintptr_t)Y % 16 == 0) &&
                  (getenv("FMX_TS_V1") == nullptr);
  const int V = v2 ? 2 : 1;
  dim3 grid((unsigned)ceil_div(A, TS_BLOCK * V), (unsigned)F);
  void* args[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&W, (void*)&present};
  if ((op == FMX_TS_DIFF || op == FMX_TS_DELAY) && W < 0) {
    grid = dim3((unsigned)ceil_div(A, TS_BLOCK), (unsigned)F);
    int K = -W;
    size_t lds = (size_t)2 * K * TS_BLOCK * sizeof(double);
    const void* k = op == FMX_TS_DIFF ? (const void*)k_ts_lead<FMX_TS_DIFF> : (const void*)k_ts_lead<FMX_TS_DELAY>;
    void* largs[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&K, (void*)&present};
    return launch_ring(k, grid, lds, st, largs);
  }
  FMX_ARG(W >= 1, "window must be >= 1");
  if (!present && op != FMX_TS_BACKFILL && getenv("FMX_TS_LDS") == nullptr) {
    const void* kr = ts_reg_kernel(op, W);
    if (kr) {
      void* rargs[] = {(void*)&X, (void*)&Y, (void*)&F, (void*)&D, (void*)&A, (void*)&ld};
      FMX_HIP(hipLaunchKernel(kr, dim3((unsigned)ceil_div(F * A, 256)), dim3(256), rargs, 0, st));
      return FMX_OK;
    }
    // other windows: the leaving value is re-read instead of kept in a ring
    const void* kl = op == FMX_TS_SUM ? (const void*)k_ts_rl<FMX_TS_SUM, 8>
                   : op == FMX_TS_MEAN ? (const void*)k_ts_rl<FMX_TS_MEAN, 8>
                   : op == FMX_TS_STD ? (const void*)k_ts_rl<FMX_TS_STD, 8>
                   : op == FMX_TS_VAR ? (const void*)k_ts_rl<FMX_TS_VAR, 8>
                   : op == FMX_TS_ZSCORE ? (const void*)k_ts_rl<FMX_TS_ZSCORE, 8> : nullptr;
    if (kl && W >= 1) {
      void* rargs[] = {(void*)&X, (void*)&Y, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&W};
      FMX_HIP(hipLaunchKernel(kl, dim3((unsigned)ceil_div(F * A, 256)), dim3(256), rargs, 0, st));
      return FMX_OK;
    }
  }
  size_t lds = (op == FMX_TS_BACKFILL) ? 0 : (size_t)W * TS_BLOCK * V * sizeof(double);
  const void* k = nullptr;
#define FMX_TSK(O) (V == 2 ? (const void*)k_ts<O, 2> : (const void*)k_ts<O, 1>)
  switch (op) {
    case FMX_TS_SUM: k = FMX_TSK(FMX_TS_SUM); break;
    case FMX_TS_MEAN: k = FMX_TSK(FMX_TS_MEAN); break;
    case FMX_TS_STD: k = FMX_TSK(FMX_TS_STD); break;
    case FMX_TS_VAR: k = FMX_TSK(FMX_TS_VAR); break;
    case FMX_TS_ZSCORE: k = FMX_TSK(FMX_TS_ZSCORE); break;
    case FMX_TS_RANK: k = FMX_TSK(FMX_TS_RANK); break;
    case FMX_TS_DECAY: k = FMX_TSK(FMX_TS_DECAY); break;
    case FMX_TS_DIFF: k = FMX_TSK(FMX_TS_DIFF); break;
    case FMX_TS_DELAY: k = FMX_TSK(FMX_TS_DELAY); break;
    default: k = FMX_TSK(FMX_TS_BACKFILL); break;
  }
#undef FMX_TSK
  return launch_ring(k, grid, lds, st, args);
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
    FMX_HIP(hipLaunchKernel((const void*)k_ts_set<20, 10, 5>, dim3((unsigned)ceil_div(F * A, 256)), dim3(256), args,
                            0, as_stream(stream)));
    return FMX_OK;
  }
  // other windows / ragged panels: one single-op pass per requested output
  const int32_t ops[5] = {FMX_TS_MEAN, FMX_TS_STD, FMX_TS_ZSCORE, FMX_TS_RANK, FMX_TS_DECAY};
  for (int k = 0; k < 5; ++k) {
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
  if (!present && getenv("FMX_TS_LDS") == nullptr) {   // dense: leaving values re-read
    void* rargs[] = {(void*)&X, (void*)&Ycol, (void*)&Out, (void*)&F, (void*)&D, (void*)&A, (void*)&ld,
                     (void*)&y_fstride, (void*)&W};
    // two dates of the four streams in flight: 116 VGPRs, 4 waves/SIMD (four dates: 154
    // VGPRs, 3 waves, 160 vs 156 ms at C5; eight: 180 ms; forcing 4-5 waves spills)
    const void* kc = (const void*)k_ts_corr_rl<2>;
    FMX_HIP(hipLaunchKernel(kc, dim3((unsigned)ceil_div(F * A, 256)), dim3(256), rargs, 0, as_stream(stream)));
    return FMX_OK;
  }
  dim3 grid((unsigned)ceil_div(A, TS_BLOCK), (unsigned)F);
  size_t lds = (size_t)2 * W * TS_BLOCK * sizeof(double);
  void* args[] = {(void*)&X, (void*)&Ycol, (void*)&Out, (void*)&D, (void*)&A, (void*)&ld,
                  (void*)&y_fstride, (void*)&W, (void*)&present};
  return launch_ring((const void*)k_ts_corr, grid, lds, as_stream(stream), args);
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
  FMX_HIP(hipLaunchKernel((const void*)k_ts_cvf_rl<8>, dim3((unsigned)ceil_div(F * A, 256)), dim3(256), args, 0,
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
  dim3 grid((unsigned)ceil_div(A, TS_BLOCK), 1);
  size_t lds = (size_t)2 * W * TS_BLOCK * sizeof(double);
  void* args[] = {(void*)&Yv, (void*)&Xv, (void*)&valid, (void*)&Out, (void*)&D, (void*)&A, (void*)&ld,
                  (void*)&W, (void*)&rt};
  return launch_ring((const void*)k_ts_regression, grid, lds, as_stream(stream), args);
}
