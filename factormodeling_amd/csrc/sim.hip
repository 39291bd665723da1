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
// the next date's row of Wout; with a presence mask it is fmx_ts_op(DELAY, 1) over the mask.
#include <hip/hip_runtime.h>
#include <cmath>
#include "../../include/fmx.h"
#include "fmx_common.hpp"

namespace fmx {

constexpr int SIM_BLOCK = 256;

__global__ void __launch_bounds__(SIM_BLOCK)
k_trade_equal(const double* __restrict__ X, const uint8_t* __restrict__ present, double* __restrict__ W,
              double* __restrict__ Wshift, double* __restrict__ counts, int64_t D, int64_t A, double pct) {
  extern __shared__ double sx[];  // [A]
  __shared__ int s_npos, s_nneg;
  __shared__ unsigned s_hist[512];
  __shared__ uint64_t s_prefix[2], s_mask[2];
  __shared__ unsigned s_krem[2];
  const int64_t d = blockIdx.x;
  const double* x = X + d * A;
  const uint8_t* p = present ? present + d * A : nullptr;
  double* w = W + d * A;
  if (threadIdx.x == 0) { s_npos = 0; s_nneg = 0; }
  __syncthreads();
  int np = 0, nn = 0;
  for (int64_t a = threadIdx.x; a < A; a += SIM_BLOCK) {
    const double v = (!p || p[a]) ? x[a] : __builtin_nan("");
    sx[a] = v;
    np += v > 0.0;
    nn += v < 0.0;
  }
  atomicAdd(&s_npos, np);
  atomicAdd(&s_nneg, nn);
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
  if (threadIdx.x == 0) {
    counts[2 * d] = (double)kl;
    counts[2 * d + 1] = (double)ks;
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
  return fmx_ts_op(FMX_TS_DELAY, Wraw, Wout, 1, D, A, A, 1, present, stream);
}
