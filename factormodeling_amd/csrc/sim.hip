// Daily trade list, method 'equal' (portfolio_simulation.py:96-170).
//
// Per date (one workgroup per [A] row, staged once in LDS): pos = x > 0, neg = x < 0 over
// the present cells (NaN compares false); if either leg is empty the day is flat (0.0 on
// present cells, counts 0/0, :108-116).  Else k_long = max(floor(n_pos * pct), 1) and
// k_short likewise (:158-159); the k_long largest positives get 1.0 / k_long and the
// k_short smallest negatives -1.0 / k_short -- exactly what _normalize_legs (:250-262)
// computes from the 1.0 / -1.0 markers, since the leg sums are the exact integers k.
// An element's place in its leg is its count of strictly better elements plus the equal
// ones at lower asset index; exact ties at the k-th value are resolved that way (the
// reference uses numpy's unstable quicksort there: implementation-defined order).
// The per-symbol shift(1) (:151-152) is fmx_ts_op(DELAY, 1) over the same presence mask.
#include <hip/hip_runtime.h>
#include <cmath>
#include "../../include/fmx.h"
#include "fmx_common.hpp"

namespace fmx {

constexpr int SIM_BLOCK = 256;
constexpr int SIM_PER = 4;  // elements ranked per lane per pass (LDS reads amortised)

__global__ void __launch_bounds__(SIM_BLOCK)
k_trade_equal(const double* __restrict__ X, const uint8_t* __restrict__ present, double* __restrict__ W,
              double* __restrict__ counts, int64_t A, double pct) {
  extern __shared__ double sx[];  // [A]
  __shared__ int s_npos, s_nneg;
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
  const double wl = flat ? 0.0 : 1.0 / (double)kl;
  const double wsh = flat ? 0.0 : -1.0 / (double)ks;
  for (int64_t a0 = (int64_t)threadIdx.x * SIM_PER; a0 < A; a0 += (int64_t)SIM_BLOCK * SIM_PER) {
    double v[SIM_PER];
    int better[SIM_PER];
#pragma unroll
    for (int u = 0; u < SIM_PER; ++u) {
      v[u] = a0 + u < A ? sx[a0 + u] : __builtin_nan("");
      better[u] = 0;
    }
    if (!flat) {
      // all lanes read the same sx[b]: LDS broadcast
      for (int64_t b = 0; b < A; ++b) {
        const double y = sx[b];
#pragma unroll
        for (int u = 0; u < SIM_PER; ++u) {
          const bool tie_before = (y == v[u]) && (b < a0 + u);
          better[u] += (v[u] > 0.0) ? ((y > v[u]) | tie_before) : ((y < v[u]) | tie_before);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < SIM_PER; ++u) {
      const int64_t a = a0 + u;
      if (a >= A) break;
      double out;
      if (p && !p[a]) out = __builtin_nan("");
      else if (flat) out = 0.0;
      else if (v[u] > 0.0 && better[u] < kl) out = wl;
      else if (v[u] < 0.0 && better[u] < ks) out = wsh;
      else out = 0.0;
      w[a] = out;
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
  k_trade_equal<<<(unsigned)D, SIM_BLOCK, lds, as_stream(stream)>>>(X, present, Wraw,
                                                                                           counts, A, pct);
  FMX_LAUNCH_CHECK("k_trade_equal");
  return fmx_ts_op(FMX_TS_DELAY, Wraw, Wout, 1, D, A, A, 1, present, stream);
}
