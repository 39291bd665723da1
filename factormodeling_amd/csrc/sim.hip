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

namespace fmx {

constexpr int SIM_BLOCK = 256;

__global__ void __launch_bounds__(SIM_BLOCK)
k_trade_equal(const double* __restrict__ X, const uint8_t* __restrict__ present, double* __restrict__ W,
              double* __restrict__ Wshift, double* __restrict__ counts, int64_t D, int64_t A, double pct) {
  extern __shared__ double sx[];  // [A]
  __shared__ int s_npos, s_nneg, s_npres;
  __shared__ unsigned s_hist[512];
  __shared__ uint64_t s_prefix[2], s_mask[2];
  __shared__ unsigned s_krem[2];
  const int64_t d = blockIdx.x;
  const double* x = X + d * A;
  const uint8_t* p = present ? present + d * A : nullptr;
  double* w = W + d * A;
  if (threadIdx.x == 0) { s_npos = 0; s_nneg = 0; s_npres = 0; }
  __syncthreads();
  int np = 0, nn = 0, npr = 0;
  for (int64_t a = threadIdx.x; a < A; a += SIM_BLOCK) {
    const bool pr = !p || p[a];
    npr += pr;
    const double v = pr ? x[a] : __builtin_nan("");
    sx[a] = v;
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
        const double v = sx[a];
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
  for (int64_t a = threadIdx.x; a < A; a += SIM_BLOCK) {
    const double v = sx[a];
    double out = 0.0;
    if (p && !p[a]) {
      out = __builtin_nan("");
    } else if (!flat && (v > 0.0 || v < 0.0)) {
      const bool lg = v > 0.0;
      const uint64_t k = (uint64_t)__double_as_longlong(lg ? v : -v);
      const uint64_t t = lg ? t0 : t1;
      bool sel = k > t;
      if (k == t) {  // exact tie at the k-th key: lowest asset indices first
        unsigned before = 0;
        for (int64_t b = 0; b < a; ++b) before += (sx[b] == v);
        sel = before < (lg ? r0 : r1);
      }
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

}  // namespace fmx

using namespace fmx;

extern "C" fmx_status fmx_trade_equal(const double* X, const uint8_t* present, double* Wraw, double* Wout,
                                      double* counts, int64_t D, int64_t A, double pct, void* stream) {
  FMX_ARG(X && Wraw && Wout && counts && D >= 0 && A >= 0, "bad args");
  FMX_ARG(Wraw != Wout && Wraw != X, "Wraw must not alias X or Wout");
  FMX_ARG(A <= 16384, "trade list stages one date row in LDS: A <= 16384");
  FMX_ARG(pct >= 0.0, "pct must be >= 0");
  if (D == 0 || A == 0) return FMX_OK;
  const size_t lds = (size_t)A * sizeof(double);
  if (lds > 64 * 1024)
    FMX_HIP(hipFuncSetAttribute((const void*)k_trade_equal, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  // dense: the kernel writes the shifted book too; ragged: shift over each symbol's rows
  k_trade_equal<<<(unsigned)D, SIM_BLOCK, lds, as_stream(stream)>>>(X, present, Wraw, present ? nullptr : Wout,
                                                                    counts, D, A, pct);
  FMX_LAUNCH_CHECK("k_trade_equal");
  if (!present) return FMX_OK;
  dim3 g((unsigned)ceil_div(A, 256), (unsigned)ceil_div(D, SHIFT_SEG));
  k_shift_rows<<<g, 256, 0, as_stream(stream)>>>(Wraw, Wout, D, A);
  FMX_LAUNCH_CHECK("k_shift_rows");
  return FMX_OK;
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
