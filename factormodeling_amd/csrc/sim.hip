// Daily trade list, method 'equal' (portfolio_simulation.py:96-170).
//
// Per date (one workgroup per [A] row, staged once in LDS): pos = x > 0, neg = x < 0 over
// the present cells (NaN compares false); if either leg is empty the day is flat (0.0 on
// present cells, counts 0/0, :108-116).  Else k_long = max(floor(n_pos * pct), 1) and
// k_short likewise (:158-159); the k_long largest positives get 1.0 / k_long and the
// k_short smallest negatives -1.0 / k_short -- exactly what _normalize_legs (:250-262)
// computes from the 1.0 / -1.0 markers, since the leg sums are the exact integers k.
// The k-th extreme key of each leg is found by an 8-pass LDS radix select (O(A) per row);
// elements beyond it are selected, and exact ties AT it go to the lowest asset indices
// (the reference uses numpy's unstable quicksort there: implementation-defined order).
// The per-symbol shift(1) (:151-152): on a dense panel the kernel also writes each row into
// the next date's row of Wout; with a presence mask k_shift_rows walks each symbol's rows.
#include <hip/hip_runtime.h>
#include <cmath>
#include <algorithm>
#include "../../include/fmx.h"
#include "fmx_common.hpp"
#include "rowkit.hpp"

namespace fmx {

constexpr int SIM_BLOCK = 256;

// STAGED: the row lives in LDS (A <= 20,480); else every pass re-reads it from HBM / L2
// (the cell value, masked by presence, is recomputed on the fly) -- any row length.
template <bool STAGED>
__global__ void __launch_bounds__(SIM_BLOCK)
k_trade_equal(const double* __restrict__ X, const uint8_t* __restrict__ present, double* __restrict__ W,
              double* __restrict__ Wshift, double* __restrict__ counts, int64_t D, int64_t A, double pct,
              int nan_absent) {
  extern __shared__ double sx[];  // [A] (STAGED)
  __shared__ int s_npos, s_nneg, s_npres;
  __shared__ unsigned s_hist[512];
  __shared__ uint64_t s_prefix[2], s_mask[2];
  __shared__ unsigned s_krem[2], s_tie[2];
  __shared__ unsigned s_wt[2][SIM_BLOCK / 64];
  const int64_t d = blockIdx.x, mgr = blockIdx.y;   // managers batched along y
  X += mgr * D * A;
  W += mgr * D * A;
  if (Wshift) Wshift += mgr * D * A;
  counts += mgr * D * 2;
  const double* x = X + d * A;
  const uint8_t* p = present ? present + d * A : nullptr;
  double* w = W + d * A;
  auto cell = [&](int64_t a) {
    if (STAGED) return sx[a];
    const double xv = x[a];
    return ((!p || p[a]) && (!nan_absent || xv == xv)) ? xv : __builtin_nan("");
  };
  if (threadIdx.x == 0) { s_npos = 0; s_nneg = 0; s_npres = 0; }
  __syncthreads();
  int np = 0, nn = 0, npr = 0;
  for (int64_t a = threadIdx.x; a < A; a += SIM_BLOCK) {
    // nan_absent: a NaN cell is no row (multi_manager.py:44 feeds factors_df[fac].dropna())
    const bool pr = (!p || p[a]) && (!nan_absent || x[a] == x[a]);
    npr += pr;
    const double v = pr ? x[a] : __builtin_nan("");
    if (STAGED) sx[a] = v;
    np += v > 0.0;
    nn += v < 0.0;
  }
  atomicAdd(&s_npos, np);
  atomicAdd(&s_nneg, nn);
  atomicAdd(&s_npres, npr);
  __syncthreads();
  const int npos = s_npos, nneg = s_nneg;
  const bool flat = npos == 0 || nneg == 0;
  const int kl = flat ? 0 : max((int)floor((double)npos * pct), 1);
  const int ks = flat ? 0 : max((int)floor((double)nneg * pct), 1);
  // pct > 1: iloc[:k] keeps the whole leg, and the leg then sums to its size
  const int nl = min(kl, npos), ns = min(ks, nneg);
  const double wl = flat ? 0.0 : 1.0 / (double)nl;
  const double wsh = flat ? 0.0 : -1.0 / (double)ns;
  if (threadIdx.x == 0) {
    s_prefix[0] = s_prefix[1] = 0;
    s_mask[0] = s_mask[1] = 0;
    s_krem[0] = (unsigned)nl;
    s_krem[1] = (unsigned)ns;
    s_tie[0] = s_tie[1] = 0;
  }
  __syncthreads();
  // k-th extreme of each leg by an 8-pass radix select over the 64-bit keys (positive
  // doubles order like their bit patterns): leg 0 keys = bits(v) for v > 0, leg 1 keys =
  // bits(-v) for v < 0; both legs want their k-th LARGEST key.
  if (!flat) {
    for (int pass = 0; pass < 8; ++pass) {
      const int shift = 56 - 8 * pass;
      for (int i = threadIdx.x; i < 512; i += SIM_BLOCK) s_hist[i] = 0;
      __syncthreads();
      const uint64_t m0 = s_mask[0], m1 = s_mask[1], p0 = s_prefix[0], p1 = s_prefix[1];
      for (int64_t a = threadIdx.x; a < A; a += SIM_BLOCK) {
        const double v = cell(a);
        if (v > 0.0) {
          const uint64_t k = (uint64_t)__double_as_longlong(v);
          if ((k & m0) == p0) atomicAdd(&s_hist[(k >> shift) & 255], 1u);
        } else if (v < 0.0) {
          const uint64_t k = (uint64_t)__double_as_longlong(-v);
          if ((k & m1) == p1) atomicAdd(&s_hist[256 + ((k >> shift) & 255)], 1u);
        }
      }
      __syncthreads();
      if (threadIdx.x < 128) {  // wave w walks leg w's bins from the top, 4 bins per lane
        const int leg = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const unsigned* h = s_hist + 256 * leg + 252 - 4 * lane;  // bins 255-4l .. 252-4l
        const unsigned c3 = h[3], c2 = h[2], c1 = h[1], c0 = h[0];
        const unsigned mine = c3 + c2 + c1 + c0;
        unsigned incl = mine;  // inclusive prefix over lanes (lane 0 = top bins)
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const unsigned o = __shfl_up(incl, off, 64);
          if (lane >= off) incl += o;
        }
        const unsigned need = s_krem[leg];
        const uint64_t hit = __ballot(incl >= need);
        const int first = hit ? __ffsll((unsigned long long)hit) - 1 : 63;
        if (lane == first) {
          unsigned cum = incl - mine;
          int bin = 255 - 4 * lane;
          const unsigned cs[4] = {c3, c2, c1, c0};
          int j = 0;
          for (; j < 3; ++j) {
            if (cum + cs[j] >= need) break;
            cum += cs[j];
          }
          bin -= j;
          if (pass == 7) s_tie[leg] = cs[j];   // #keys equal to the k-th key
          s_krem[leg] = need - cum;
          s_prefix[leg] |= (uint64_t)bin << shift;
          s_mask[leg] |= (uint64_t)255 << shift;
        }
      }
      __syncthreads();
    }
  }
  const uint64_t t0 = s_prefix[0], t1 = s_prefix[1];
  const unsigned r0 = s_krem[0], r1 = s_krem[1];
  // Exact ties at a leg's k-th key go to the lowest asset indices: when a leg has more
  // keys equal to its k-th than it still needs, each tied element's index among them comes
  // from a block-wide scan (wave ballots + per-wave totals), chunk by chunk in asset order.
  const bool scan = !flat && (s_tie[0] > r0 || s_tie[1] > r1);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned base0 = 0, base1 = 0;                      // ties in earlier chunks
  for (int64_t a0 = 0; a0 < A; a0 += SIM_BLOCK) {
    const int64_t a = a0 + threadIdx.x;
    const bool in = a < A;
    const double v = in ? cell(a) : __builtin_nan("");
    const bool lg = v > 0.0;
    const uint64_t k = (uint64_t)__double_as_longlong(lg ? v : -v);
    const bool tie0 = !flat && lg && k == t0, tie1 = !flat && v < 0.0 && k == t1;
    unsigned before = 0;
    if (scan) {
      const uint64_t b0 = __ballot(tie0), b1 = __ballot(tie1);
      const uint64_t lt = (1ull << lane) - 1ull;
      if (lane == 0) { s_wt[0][wid] = __popcll(b0); s_wt[1][wid] = __popcll(b1); }
      __syncthreads();
      unsigned off0 = 0, off1 = 0, tot0 = 0, tot1 = 0;
#pragma unroll
      for (int q = 0; q < SIM_BLOCK / 64; ++q) {
        const unsigned c0 = s_wt[0][q], c1 = s_wt[1][q];
        off0 += q < wid ? c0 : 0u;
        off1 += q < wid ? c1 : 0u;
        tot0 += c0;
        tot1 += c1;
      }
      __syncthreads();                                // s_wt reused by the next chunk
      before = tie0 ? base0 + off0 + (unsigned)__popcll(b0 & lt) : base1 + off1 + (unsigned)__popcll(b1 & lt);
      base0 += tot0;
      base1 += tot1;
    }
    if (!in) continue;
    double out = 0.0;
    if ((p && !p[a]) || (nan_absent && v != v)) {
      out = __builtin_nan("");
    } else if (!flat && (v > 0.0 || v < 0.0)) {
      const uint64_t t = lg ? t0 : t1;
      bool sel = k > t;
      if (k == t) sel = scan ? before < (lg ? r0 : r1) : true;
      if (sel) out = lg ? wl : wsh;
    }
    w[a] = out;
    if (Wshift) {  // dense panel: shift(1) per symbol is the next date's row
      if (d + 1 < D) Wshift[(d + 1) * A + a] = out;
      if (d == 0) Wshift[a] = __builtin_nan("");
    }
  }
  if (threadIdx.x == 0) {  // a date with no rows has no counts row in the reference: NaN
    counts[2 * d] = s_npres ? (double)kl : __builtin_nan("");
    counts[2 * d + 1] = s_npres ? (double)ks : __builtin_nan("");
  }
}

// Per-symbol shift(1) over present rows of a same-day book W (present cells are never NaN
// in it, absent ones always are), split into date segments of SHIFT_SEG so the grid fills
// the chip: each (segment, asset) lane first looks back for the last present value before
// its segment, then walks its dates.
constexpr int SHIFT_SEG = 64;
__global__ void k_shift_rows(const double* __restrict__ W, double* __restrict__ out, int64_t D, int64_t A) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= A) return;
  W += (int64_t)blockIdx.z * D * A;               // managers batched along z
  out += (int64_t)blockIdx.z * D * A;
  const int64_t d0 = (int64_t)blockIdx.y * SHIFT_SEG;
  const int64_t d1 = d0 + SHIFT_SEG < D ? d0 + SHIFT_SEG : D;
  double last = __builtin_nan("");
  for (int64_t d = d0 - 1; d >= 0; --d) {
    const double v = W[d * A + a];
    if (v == v) { last = v; break; }
  }
  for (int64_t d = d0; d < d1; ++d) {
    const double v = W[d * A + a];
    out[d * A + a] = (v == v) ? last : v;
    if (v == v) last = v;
  }
}

// multi_manager.compute_multimanager_weights (multi_manager.py:32-81): per weight date j
// (date index wdate[j]) and asset a, fold the manager books in factor_weights column order:
// acc = 0.0; acc += Wf[f][d][a] * fw[j][c] for columns with a manager (colmap >= 0), a
// nonzero weight and rows on that date (counts not NaN), NaN products filled with 0
// (Series.add(fill_value=0), :63); counts fold fw * count likewise (:64-65).
__global__ void k_mm_combine(const double* __restrict__ Wf, const double* __restrict__ cnt,
                             const double* __restrict__ fw, const int32_t* __restrict__ colmap,
                             const int32_t* __restrict__ wdate, double* __restrict__ out,
                             double* __restrict__ out_counts, int64_t Fw, int64_t D, int64_t A) {
  const int64_t j = blockIdx.y;
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t d = wdate[j];
  double acc = 0.0, lc = 0.0, sc = 0.0;
  for (int64_t c = 0; d >= 0 && c < Fw; ++c) {  // d < 0: a date no manager has
    const int f = colmap[c];
    const double w = fw[j * Fw + c];
    if (f < 0 || w == 0.0) continue;
    const double k0 = cnt[((int64_t)f * D + d) * 2];
    if (k0 != k0) continue;  // xs(date) KeyError: manager has no rows that day
    if (a < A) {
      const double p = Wf[((int64_t)f * D + d) * A + a] * w;
      if (p == p) acc = acc + p;
    }
    lc = lc + w * k0;
    sc = sc + w * cnt[((int64_t)f * D + d) * 2 + 1];
  }
  if (a < A) out[j * A + a] = acc;
  if (a == 0) {
    out_counts[2 * j] = lc;
    out_counts[2 * j + 1] = sc;
  }
}

// ------------------------------------------------------------------------------------
// Daily trade list, method 'linear' (portfolio_simulation.py:172-181): weights = the
// signal on its positive / negative cells, _normalize_legs (:250-262) and
// _cap_and_redistribute (:264-313) with max_iter 10, tol 1e-6.  One workgroup per date;
// thread t holds the row cells t + k*LIN_NT in registers.  Every pandas sum the reference
// takes -- w_pos.sum() over the date's n rows (zeros included), capped[capped > 0].sum(),
// uncapped_long.sum(), ... -- is numpy's pairwise sum over that subset in symbol order, so
// each subset is compacted into LDS (ballot prefix per register chunk) and summed with
// the numpy schedule for its length (rowkit.hpp): the weights are bit-identical.  pandas
// clip is where(x >= lo, x, lo) then where(x <= hi, x, hi).
constexpr int LIN_NT = 1024;
constexpr int LIN_NW = LIN_NT / 64;

// Compact the cells whose bit k of `flags` is set, in asset order, into sub[0..m); all
// threads get m.  wtot: EMAX * LIN_NW ints of scratch.
template <int EMAX>
__device__ int lin_compact(const double* v, uint32_t flags, double* sub, int* wtot) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int pre[EMAX];
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const uint64_t b = __ballot((flags >> k) & 1u);
    pre[k] = __popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0) wtot[k * LIN_NW + wid] = __popcll(b);
  }
  __syncthreads();
  if (wid == 0) {                       // exclusive scan over (chunk, wave) in asset order
    constexpr int N = EMAX * LIN_NW, PER = (N + 63) / 64;
    int loc[PER], sum = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) { const int i = lane * PER + j; loc[j] = i < N ? wtot[i] : 0; sum += loc[j]; }
    int incl = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) { const int u = __shfl_up(incl, o, 64); if (lane >= o) incl += u; }
    int run = incl - sum;
#pragma unroll
    for (int j = 0; j < PER; ++j) { const int i = lane * PER + j; if (i < N) wtot[i] = run; run += loc[j]; }
    if (lane == 63) wtot[N] = incl;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < EMAX; ++k)
    if ((flags >> k) & 1u) sub[wtot[k * LIN_NW + wid] + pre[k]] = v[k];
  const int m = wtot[EMAX * LIN_NW];
  __syncthreads();
  return m;
}

template <int EMAX>
__device__ double lin_sum(const double* v, uint32_t flags, double* sub, int* wtot, PwTable pw, double* nodes,
                          int* iscr) {
  const int m = lin_compact<EMAX>(v, flags, sub, wtot);
  int cnt;
  return block_pw_sum_w0<LIN_NT>([&](int i) { return sub[i]; }, [](int) { return 0; }, pw.get(m), nodes, iscr,
                                 &cnt);
}

template <int EMAX>
__global__ void __launch_bounds__(LIN_NT)
k_trade_linear(const double* __restrict__ X, const uint8_t* __restrict__ present, double* __restrict__ W,
               double* __restrict__ Wshift, double* __restrict__ counts, int64_t D, int64_t A, double mw,
               PwTable pw, int nan_absent) {
  extern __shared__ double sub[];                 // [A] compacted subset
  __shared__ double nodes[2 * (16384 / 64) + 8];
  __shared__ int iscr[LIN_NW + 2];
  __shared__ int wtot[EMAX * LIN_NW + 1];
  const int t = threadIdx.x;
  const int64_t d = blockIdx.x, mgr = blockIdx.y;   // managers batched along y
  X += mgr * D * A;
  W += mgr * D * A;
  if (Wshift) Wshift += mgr * D * A;
  counts += mgr * D * 2;
  const double* x = X + d * A;
  const uint8_t* p = present ? present + d * A : nullptr;
  double w[EMAX];
  uint32_t pm = 0, fpos = 0, fneg = 0;
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t a = t + (int64_t)k * LIN_NT;
    const double xv = a < A ? x[a] : 0.0;
    const bool pr = a < A && (!p || p[a]) && (!nan_absent || xv == xv);
    const double v = pr ? xv : 0.0;
    pm |= (uint32_t)pr << k;
    fpos |= (uint32_t)(pr && v > 0.0) << k;
    fneg |= (uint32_t)(pr && v < 0.0) << k;
    w[k] = (pr && (v > 0.0 || v < 0.0)) ? v : 0.0;  // weights[pos.index] = pos, [neg.index] = neg
  }
  int c3[3] = {(int)__popc(pm), (int)__popc(fpos), (int)__popc(fneg)};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c3[i] += __shfl_xor(c3[i], o);
  }
  if ((t & 63) == 0) { iscr[t >> 6] = c3[1]; wtot[t >> 6] = c3[2]; }
  __syncthreads();
  int npos = 0, nneg = 0;
  for (int i = 0; i < LIN_NW; ++i) { npos += iscr[i]; nneg += wtot[i]; }
  const bool anyrow = __syncthreads_or(pm != 0);
  const bool flat = npos == 0 || nneg == 0;
  if (!flat) {
    // _normalize_legs: w_pos = clip(lower=0), w_neg = clip(upper=0), sums over all n rows
    double wp[EMAX], wn[EMAX];
#pragma unroll
    for (int k = 0; k < EMAX; ++k) { wp[k] = w[k] >= 0.0 ? w[k] : 0.0; wn[k] = w[k] <= 0.0 ? w[k] : 0.0; }
    const double sp = lin_sum<EMAX>(wp, pm, sub, wtot, pw, nodes, iscr);
    const double sn = lin_sum<EMAX>(wn, pm, sub, wtot, pw, nodes, iscr);
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const double a = sp > 0.0 ? wp[k] / sp : wp[k];
      const double b = sn < 0.0 ? wn[k] / -sn : wn[k];
      w[k] = a + b;
    }
    // _cap_and_redistribute(max_weight, max_iter=10, tol=1e-6)
    const double tol = 1e-6;
    for (int it = 0; it < 10; ++it) {
      double c[EMAX];
      uint32_t fcp = 0, fcn = 0, ful = 0, fus = 0;
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
        double v = w[k] >= -mw ? w[k] : -mw;
        v = v <= mw ? v : mw;
        c[k] = v;
        const uint32_t pr = (pm >> k) & 1u;
        fcp |= (pr & (uint32_t)(v > 0.0)) << k;
        fcn |= (pr & (uint32_t)(v < 0.0)) << k;
        ful |= (pr & (uint32_t)(w[k] > 0.0 && v < mw)) << k;
        fus |= (pr & (uint32_t)(w[k] < 0.0 && v > -mw)) << k;
      }
      const double le = 1.0 - lin_sum<EMAX>(c, fcp, sub, wtot, pw, nodes, iscr);
      const double se = -1.0 - lin_sum<EMAX>(c, fcn, sub, wtot, pw, nodes, iscr);
      const bool any_ul = __syncthreads_or(ful != 0), any_us = __syncthreads_or(fus != 0);
      if ((fabs(le) < tol && fabs(se) < tol) || (!any_ul && !any_us)) break;
      if (any_ul && fabs(le) > tol) {
        const double su = lin_sum<EMAX>(c, ful, sub, wtot, pw, nodes, iscr);
#pragma unroll
        for (int k = 0; k < EMAX; ++k)
          if ((ful >> k) & 1u) c[k] = c[k] + le * (c[k] / su);
      }
      if (any_us && fabs(se) > tol) {
        const double su = lin_sum<EMAX>(c, fus, sub, wtot, pw, nodes, iscr);
#pragma unroll
        for (int k = 0; k < EMAX; ++k)
          if ((fus >> k) & 1u) c[k] = c[k] + se * (c[k] / su);
      }
#pragma unroll
      for (int k = 0; k < EMAX; ++k) w[k] = c[k];
    }
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      double v = w[k] >= -mw ? w[k] : -mw;
      w[k] = v <= mw ? v : mw;
    }
  }
  double* wr = W + d * A;
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t a = t + (int64_t)k * LIN_NT;
    if (a >= A) continue;
    const double out = ((pm >> k) & 1u) ? (flat ? 0.0 : w[k]) : __builtin_nan("");
    wr[a] = out;
    if (Wshift) {
      if (d + 1 < D) Wshift[(d + 1) * A + a] = out;
      if (d == 0) Wshift[a] = __builtin_nan("");
    }
  }
  if (t == 0) {                                   // counts (len(pos), len(neg)); NaN: no rows
    counts[2 * d] = anyrow ? (flat ? 0.0 : (double)npos) : __builtin_nan("");
    counts[2 * d + 1] = anyrow ? (flat ? 0.0 : (double)nneg) : __builtin_nan("");
  }
}

// Trade list 'linear' on rows past 16,384 assets (k_trade_linear holds a row in registers):
// the same operations in the same order, with the row's weights held in its output row W
// (not registers) and each subset compacted, in asset order, into Wsub's row (the shifted
// book, written by k_shift_rows afterwards) instead of LDS.  One workgroup per (date,
// manager).  ful / fus are read off the capped weight c: for mw > 0, w > 0 && c < mw <=>
// 0 < c < mw (and w < 0 && c > -mw <=> -mw < c < 0).
__global__ void __launch_bounds__(LIN_NT)
k_trade_linear_xl(const double* __restrict__ X, const uint8_t* __restrict__ present, double* __restrict__ W,
                  double* __restrict__ Wsub, double* __restrict__ counts, int64_t D, int64_t A, double mw, PwTable pw,
                  int nan_absent) {
  __shared__ double nodes[2 * (65536 / 64) + 8];
  __shared__ int iscr[LIN_NW + 2];
  const int t = threadIdx.x;
  const int64_t d = blockIdx.x, mgr = blockIdx.y;
  const double* x = X + mgr * D * A + d * A;
  const uint8_t* p = present ? present + d * A : nullptr;
  double* w = W + mgr * D * A + d * A;
  double* sub = Wsub + mgr * D * A + d * A;
  counts += mgr * D * 2;
  auto pres = [&](int64_t a) {
    const double xv = x[a];
    return (!p || p[a]) && (!nan_absent || xv == xv);
  };
  int c3[3] = {0, 0, 0};
  for (int64_t a = t; a < A; a += LIN_NT) {
    const bool pr = pres(a);
    const double v = pr ? x[a] : 0.0;
    c3[0] += pr;
    c3[1] += pr && v > 0.0;
    c3[2] += pr && v < 0.0;
    w[a] = (pr && (v > 0.0 || v < 0.0)) ? v : 0.0;   // weights[pos.index] = pos, [neg.index] = neg
  }
  int tot[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    block_exscan<LIN_NT>(c3[i], iscr, &tot[i]);
    __syncthreads();
  }
  const int npos = tot[1], nneg = tot[2];
  const bool anyrow = tot[0] > 0;
  const bool flat = npos == 0 || nneg == 0;
  // numpy pairwise sum over the cells a < A with sel(a), of val(a), in asset order
  auto csum = [&](auto val, auto sel) {
    int m = 0;
    for (int64_t c0 = 0; c0 < A; c0 += LIN_NT) {
      const int64_t a = c0 + t;
      const bool in = a < A && sel(a);
      int n;
      const int off = block_exscan<LIN_NT>(in ? 1 : 0, iscr, &n);
      if (in) sub[m + off] = val(a);
      m += n;
      __syncthreads();
    }
    int cnt;
    return block_pw_sum_w0<LIN_NT>([&](int i) { return sub[i]; }, [](int) { return 0; }, pw.get(m), nodes, iscr,
                                   &cnt);
  };
  if (!flat) {
    // _normalize_legs: w_pos = clip(lower=0), w_neg = clip(upper=0), sums over all n rows
    const double sp = csum([&](int64_t a) { const double v = w[a]; return v >= 0.0 ? v : 0.0; }, pres);
    const double sn = csum([&](int64_t a) { const double v = w[a]; return v <= 0.0 ? v : 0.0; }, pres);
    for (int64_t a = t; a < A; a += LIN_NT) {
      const double v = w[a];
      const double wp = v >= 0.0 ? v : 0.0, wn = v <= 0.0 ? v : 0.0;
      const double aa = sp > 0.0 ? wp / sp : wp;
      const double bb = sn < 0.0 ? wn / -sn : wn;
      w[a] = aa + bb;
    }
    __syncthreads();
    // _cap_and_redistribute(max_weight, max_iter=10, tol=1e-6): w becomes c in place
    const double tol = 1e-6;
    for (int it = 0; it < 10; ++it) {
      bool ul = false, us = false;
      for (int64_t a = t; a < A; a += LIN_NT) {
        double v = w[a] >= -mw ? w[a] : -mw;
        v = v <= mw ? v : mw;
        w[a] = v;
        const bool pr = pres(a);
        ul |= pr && v > 0.0 && v < mw;
        us |= pr && v < 0.0 && v > -mw;
      }
      __syncthreads();
      const double le = 1.0 - csum([&](int64_t a) { return w[a]; }, [&](int64_t a) { return pres(a) && w[a] > 0.0; });
      const double se = -1.0 - csum([&](int64_t a) { return w[a]; }, [&](int64_t a) { return pres(a) && w[a] < 0.0; });
      const bool any_ul = __syncthreads_or(ul), any_us = __syncthreads_or(us);
      if ((fabs(le) < tol && fabs(se) < tol) || (!any_ul && !any_us)) break;
      auto ful = [&](int64_t a) { const double v = w[a]; return pres(a) && v > 0.0 && v < mw; };
      auto fus = [&](int64_t a) { const double v = w[a]; return pres(a) && v < 0.0 && v > -mw; };
      if (any_ul && fabs(le) > tol) {
        const double su = csum([&](int64_t a) { return w[a]; }, ful);
        for (int64_t a = t; a < A; a += LIN_NT)
          if (ful(a)) w[a] = w[a] + le * (w[a] / su);
        __syncthreads();
      }
      if (any_us && fabs(se) > tol) {
        const double su = csum([&](int64_t a) { return w[a]; }, fus);
        for (int64_t a = t; a < A; a += LIN_NT)
          if (fus(a)) w[a] = w[a] + se * (w[a] / su);
        __syncthreads();
      }
    }
  }
  for (int64_t a = t; a < A; a += LIN_NT) {
    double v = w[a] >= -mw ? w[a] : -mw;
    v = v <= mw ? v : mw;
    w[a] = pres(a) ? (flat ? 0.0 : v) : __builtin_nan("");
  }
  if (t == 0) {                                   // counts (len(pos), len(neg)); NaN: no rows
    counts[2 * d] = anyrow ? (flat ? 0.0 : (double)npos) : __builtin_nan("");
    counts[2 * d + 1] = anyrow ? (flat ? 0.0 : (double)nneg) : __builtin_nan("");
  }
}

// ------------------------------------------------------------------------------------
// Simulation._daily_portfolio_returns (portfolio_simulation.py:748-797)
// on the aligned [D][A] grid (union of the weights' and returns' dates and symbols; NaN =
// a cell the reference's unstack().fillna(0) makes 0).  One workgroup per date row:
//   longs = max(w, 0), shorts = |min(w, 0)|
//   out[d][0] = sum longs * r            (long_ret_raw, :758)
//   out[d][1] = sum shorts * r           (short_ret_raw = -out[1], :759)
//   out[d][2] = sum |longs - longs_prev|  (long turnover, :761; prev = previous weights date)
//   out[d][3] = sum |shorts - shorts_prev|
//   out[d][4] = sum |d longs| * rate(cap) (long cost, :766-767; rate 1 -> 0.0025, 2 -> 0.0015,
//   out[d][5] = sum |d shorts| * rate(cap)   3 -> 0.0010, other ints as themselves, :764-765)
// wprev[d] = row of the previous weights date (-1: first weights date or not one: no diff).
// Block sums are deterministic (fixed lane/wave order); the reference sums rows with
// numpy (order differs in the last bits only).
constexpr int PNL_NT = 256;
__device__ __forceinline__ double cap_rate(double c) {
  const double ci = (c == c) ? trunc(c) : 0.0;   // fillna(0).astype(int)
  return ci == 1.0 ? 0.0025 : ci == 2.0 ? 0.0015 : ci == 3.0 ? 0.0010 : ci;
}
__device__ __forceinline__ double nz(double v) { return v == v ? v : 0.0; }

template <int N>
__device__ __forceinline__ void pnl_block_sum(double* v, double* scr) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[i] += __shfl_xor(v[i], o);
    if (lane == 0) scr[wid * N + i] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double t = 0.0;
    for (int w = 0; w < PNL_NT / 64; ++w) t += scr[w * N + i];
    v[i] = t;
  }
}

__global__ void __launch_bounds__(PNL_NT)
k_pnl_daily(const double* __restrict__ W, const double* __restrict__ R, const double* __restrict__ CAP,
            const int32_t* __restrict__ wprev, double* __restrict__ out, int64_t A) {
  __shared__ double scr[(PNL_NT / 64) * 6];
  const int64_t d = blockIdx.x;
  const int64_t pv = wprev[d];
  const double* w = W + d * A;
  const double* r = R + d * A;
  const double* wp = pv >= 0 ? W + pv * A : nullptr;
  const double* cp = CAP ? CAP + d * A : nullptr;
  double acc[6] = {0, 0, 0, 0, 0, 0};
  for (int64_t a = threadIdx.x; a < A; a += PNL_NT) {
    const double wv = nz(w[a]), rv = nz(r[a]);
    const double l = wv > 0.0 ? wv : 0.0, sh = wv < 0.0 ? -wv : 0.0;
    acc[0] += l * rv;
    acc[1] += sh * rv;
    if (wp) {
      const double pw = nz(wp[a]);
      const double pl = pw > 0.0 ? pw : 0.0, ps = pw < 0.0 ? -pw : 0.0;
      const double dl = fabs(l - pl), ds = fabs(sh - ps);
      const double rate = cp ? cap_rate(cp[a]) : 0.0;
      acc[2] += dl;
      acc[3] += ds;
      acc[4] += dl * rate;
      acc[5] += ds * rate;
    }
  }
  pnl_block_sum<6>(acc, scr);
  if (threadIdx.x < 6) out[d * 6 + threadIdx.x] = acc[threadIdx.x];
}

// Per-symbol contributions (contributor=True, :790-793): column sums over the dates of
// longs * r - |d longs| * rate (and the short leg with -shorts * r).  One lane per asset.
__global__ void k_pnl_contrib(const double* __restrict__ W, const double* __restrict__ R,
                              const double* __restrict__ CAP, const int32_t* __restrict__ wprev,
                              double* __restrict__ out, int64_t D, int64_t A) {
  const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= A) return;
  double lp = 0.0, sp = 0.0, lc = 0.0, sc = 0.0;
  for (int64_t d = 0; d < D; ++d) {
    const double wv = nz(W[d * A + a]), rv = nz(R[d * A + a]);
    const double l = wv > 0.0 ? wv : 0.0, sh = wv < 0.0 ? -wv : 0.0;
    lp += l * rv;
    sp += sh * rv;
    const int64_t pv = wprev[d];
    if (pv >= 0) {
      const double pw = nz(W[pv * A + a]);
      const double pl = pw > 0.0 ? pw : 0.0, ps = pw < 0.0 ? -pw : 0.0;
      const double rate = CAP ? cap_rate(CAP[d * A + a]) : 0.0;
      lc += fabs(l - pl) * rate;
      sc += fabs(sh - ps) * rate;
    }
  }
  out[2 * a] = lp - lc;
  out[2 * a + 1] = -sp - sc;
}

// _calculate_metrics daily IC (portfolio_simulation.py:799-805): per date, pandas
// Series.corr = np.corrcoef of the pair-valid (alpha, ret) cells: two passes (means, then
// centred cross / square sums), r = (c01 / sd0) / sd1 clipped to [-1, 1]; NaN for n < 2
// or a constant side.  out[d] = (n, corr).
__global__ void __launch_bounds__(PNL_NT)
k_daily_corr(const double* __restrict__ X, const double* __restrict__ R, double* __restrict__ out, int64_t A) {
  __shared__ double scr[(PNL_NT / 64) * 3];
  const int64_t d = blockIdx.x;
  const double* x = X + d * A;
  const double* r = R + d * A;
  double s[3] = {0, 0, 0};                      // n, sum x, sum r
  for (int64_t a = threadIdx.x; a < A; a += PNL_NT) {
    const double xv = x[a], rv = r[a];
    if (xv == xv && rv == rv) { s[0] += 1.0; s[1] += xv; s[2] += rv; }
  }
  pnl_block_sum<3>(s, scr);
  const double n = s[0], mx = s[1] / n, mr = s[2] / n;
  __syncthreads();
  double c[3] = {0, 0, 0};                      // sum dx dr, dx^2, dr^2
  for (int64_t a = threadIdx.x; a < A; a += PNL_NT) {
    const double xv = x[a], rv = r[a];
    if (xv == xv && rv == rv) {
      const double dx = xv - mx, dr = rv - mr;
      c[0] += dx * dr; c[1] += dx * dx; c[2] += dr * dr;
    }
  }
  pnl_block_sum<3>(c, scr);
  if (threadIdx.x == 0) {
    double v = __builtin_nan("");
    if (n >= 2.0) {
      const double f = n - 1.0;
      const double c01 = c[0] / f, sd0 = sqrt(c[1] / f), sd1 = sqrt(c[2] / f);
      v = (c01 / sd0) / sd1;
      if (v == v) v = fmin(1.0, fmax(-1.0, v));
    }
    out[2 * d] = n;
    out[2 * d + 1] = v;
  }
}

}  // namespace fmx

using namespace fmx;

extern "C" fmx_status fmx_pnl_daily(const double* W, const double* R, const double* CAP, const int32_t* wprev,
                                    double* out, double* contrib, int64_t D, int64_t A, void* stream) {
  FMX_ARG(W && R && wprev && out && D >= 0 && A >= 0, "bad args");
  if (D == 0) return FMX_OK;
  FMX_ARG(D <= 0x7fffffffll, "too many dates");
  k_pnl_daily<<<(unsigned)D, PNL_NT, 0, as_stream(stream)>>>(W, R, CAP, wprev, out, A);
  FMX_LAUNCH_CHECK("k_pnl_daily");
  if (contrib && A > 0) {
    k_pnl_contrib<<<(unsigned)ceil_div(A, 256), 256, 0, as_stream(stream)>>>(W, R, CAP, wprev, contrib, D, A);
    FMX_LAUNCH_CHECK("k_pnl_contrib");
  }
  return FMX_OK;
}

extern "C" fmx_status fmx_daily_corr(const double* X, const double* R, double* out, int64_t D, int64_t A,
                                     void* stream) {
  FMX_ARG(X && R && out && D >= 0 && A >= 0, "bad args");
  if (D == 0) return FMX_OK;
  FMX_ARG(D <= 0x7fffffffll, "too many dates");
  k_daily_corr<<<(unsigned)D, PNL_NT, 0, as_stream(stream)>>>(X, R, out, A);
  FMX_LAUNCH_CHECK("k_daily_corr");
  return FMX_OK;
}

// Trade books of F managers [F][D][A] (F = 1: one signal), method 0 = equal, 1 = linear.
static fmx_status trade_book(int method, const double* X, const uint8_t* present, int nan_absent, double* Wraw,
                             double* Wout, double* counts, int64_t F, int64_t D, int64_t A, double pct, double mw,
                             hipStream_t st) {
  FMX_ARG(X && Wraw && Wout && counts && F >= 0 && D >= 0 && A >= 0 && A <= (1 << 20), "bad args");
  FMX_ARG(Wraw != Wout && Wraw != X, "Wraw must not alias X or Wout");
  FMX_ARG(pct >= 0.0, "pct must be >= 0");
  FMX_ARG(F <= 65535 && D <= 0x7fffffffll, "too many managers / dates");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  // rows past 16,384 assets: the linear book keeps its row in HBM (k_trade_linear_xl uses
  // Wout's row as scratch), then the shift runs as on a ragged panel
  const bool xl = A > 16384;
  FMX_ARG(!xl || method == 0 || mw > 0.0, "rows past 16384 assets: max_weight must be > 0 for 'linear'");
  const bool ragged = present || nan_absent || (xl && method == 1);
  double* ws = ragged ? nullptr : Wout;             // dense: the kernel writes the shifted book
  const size_t lds = (size_t)A * sizeof(double);
  if (method == 0) {
    const bool staged = lds <= 160 * 1024 - 8192;
    const void* k = staged ? (const void*)k_trade_equal<true> : (const void*)k_trade_equal<false>;
    const size_t dl = staged ? lds : 0;
    if (dl > 64 * 1024) FMX_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dl));
    void* args[] = {(void*)&X, (void*)&present, (void*)&Wraw, (void*)&ws, (void*)&counts, (void*)&D, (void*)&A,
                    (void*)&pct, (void*)&nan_absent};
    FMX_HIP(hipLaunchKernel(k, dim3((unsigned)D, (unsigned)F), dim3(SIM_BLOCK), args, dl, st));
  } else if (xl) {
    fmx_status e = FMX_OK;
    PwTable pw = pw_table((int)A, &e);
    if (e) return e;
    void* args[] = {(void*)&X, (void*)&present, (void*)&Wraw, (void*)&Wout, (void*)&counts, (void*)&D, (void*)&A,
                    (void*)&mw, (void*)&pw, (void*)&nan_absent};
    FMX_HIP(hipLaunchKernel((const void*)k_trade_linear_xl, dim3((unsigned)D, (unsigned)F), dim3(LIN_NT), args, 0,
                            st));
  } else {
    fmx_status e = FMX_OK;
    PwTable pw = pw_table((int)A, &e);
    if (e) return e;
    const int E = (int)ceil_div(A, LIN_NT);
    const void* k = E <= 1 ? (const void*)k_trade_linear<1> : E <= 2 ? (const void*)k_trade_linear<2>
                  : E <= 4 ? (const void*)k_trade_linear<4> : E <= 8 ? (const void*)k_trade_linear<8>
                             : (const void*)k_trade_linear<16>;
    if (lds > 64 * 1024) FMX_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    void* args[] = {(void*)&X, (void*)&present, (void*)&Wraw, (void*)&ws, (void*)&counts, (void*)&D, (void*)&A,
                    (void*)&mw, (void*)&pw, (void*)&nan_absent};
    FMX_HIP(hipLaunchKernel(k, dim3((unsigned)D, (unsigned)F), dim3(LIN_NT), args, lds, st));
  }
  if (!ragged) return FMX_OK;
  // ragged: shift over each manager's own rows (present cells are never NaN in its book)
  dim3 g((unsigned)ceil_div(A, 256), (unsigned)ceil_div(D, SHIFT_SEG), (unsigned)F);
  k_shift_rows<<<g, 256, 0, st>>>(Wraw, Wout, D, A);
  FMX_LAUNCH_CHECK("k_shift_rows");
  return FMX_OK;
}

extern "C" fmx_status fmx_shift_rows(const double* W, double* out, int64_t F, int64_t D, int64_t A, void* stream) {
  FMX_ARG(W && out && W != out && F >= 0 && D >= 0 && A >= 0 && F <= 65535, "bad args");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  dim3 g((unsigned)ceil_div(A, 256), (unsigned)ceil_div(D, SHIFT_SEG), (unsigned)F);
  k_shift_rows<<<g, 256, 0, as_stream(stream)>>>(W, out, D, A);
  FMX_LAUNCH_CHECK("k_shift_rows");
  return FMX_OK;
}

extern "C" fmx_status fmx_trade_equal(const double* X, const uint8_t* present, double* Wraw, double* Wout,
                                      double* counts, int64_t D, int64_t A, double pct, void* stream) {
  return trade_book(0, X, present, 0, Wraw, Wout, counts, 1, D, A, pct, 0.0, as_stream(stream));
}

extern "C" fmx_status fmx_trade_linear(const double* X, const uint8_t* present, double* Wraw, double* Wout,
                                       double* counts, int64_t D, int64_t A, double max_weight, void* stream) {
  return trade_book(1, X, present, 0, Wraw, Wout, counts, 1, D, A, 0.0, max_weight, as_stream(stream));
}

extern "C" fmx_status fmx_trade_books(int32_t method, const double* X, const uint8_t* present, int32_t nan_absent,
                                      double* Wraw, double* Wout, double* counts, int64_t F, int64_t D, int64_t A,
                                      double pct, double max_weight, void* stream) {
  FMX_ARG(method == 0 || method == 1, "method must be 0 (equal) or 1 (linear)");
  return trade_book(method, X, present, nan_absent, Wraw, Wout, counts, F, D, A, pct, max_weight,
                    as_stream(stream));
}

extern "C" fmx_status fmx_mm_combine(const double* Wf, const double* counts, const double* fw, const int32_t* colmap,
                                     const int32_t* wdate, double* out, double* out_counts, int64_t Fw, int64_t Dw,
                                     int64_t D, int64_t A, void* stream) {
  FMX_ARG(Wf && counts && fw && colmap && wdate && out && out_counts && Fw >= 0 && Dw >= 0 && D >= 0 && A >= 0,
          "bad args");
  if (Dw == 0) return FMX_OK;
  FMX_ARG(Dw <= 65535, "at most 65535 weight dates per call");
  dim3 grid((unsigned)ceil_div(std::max<int64_t>(A, 1), 256), (unsigned)Dw);
  k_mm_combine<<<grid, 256, 0, as_stream(stream)>>>(Wf, counts, fw, colmap, wdate, out, out_counts, Fw, D, A);
  FMX_LAUNCH_CHECK("k_mm_combine");
  return FMX_OK;
}
