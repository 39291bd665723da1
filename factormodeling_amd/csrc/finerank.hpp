// Fine-bucket ranking of one row (fp64 keys) by one workgroup.
//
// Same contract as bucketrank.hpp -- the exact average rank
//     rank = #{y < x} + (#{y == x} + 1) / 2
// from bucket counts plus an in-bucket scan -- but the buckets are cut so that almost
// every element is alone in its bucket, which removes the in-bucket scan for most
// elements and the large block-wide splitter merge:
//
//  * one wave sorts a positional sample of 64 keys in registers (xor-shuffle bitonic);
//    the sorted samples s_0..s_{ns-1} plus the row's min and max cut the key space into
//    ns + 1 coarse intervals [min, s_0), [s_0, s_1), ..., [s_{ns-1}, max] holding
//    ~A/65 members each, and ns "equal to s_j" buckets that absorb heavy ties;
//  * inside coarse interval i an element lands in fine bucket
//        sub = min(K - 1, floor((x - lo_i) * (K / (hi_i - lo_i))))
//    Every step (IEEE subtract, multiply by a non-negative constant, floor, clamp) is
//    monotone non-decreasing in x and equal keys give equal results, so bucket ids are
//    monotone in the key: correctness never depends on how well the buckets are
//    balanced, only the cost of the in-bucket scan does.
//
// Bucket id layout (K+1 ids per interval): fine bucket sub of interval i is
// i*(K+1) + sub, the equal bucket of sample j is j*(K+1) + K, so ids increase with the
// key: I_0 fine, Eq(s_0), I_1 fine, Eq(s_1), ..., Eq(s_63), I_64 fine.
#pragma once

#include "bucketrank.hpp"

namespace fmx {

constexpr int FR_S = 64;   // samples = one wave

template <int K>
struct FRG {
  static constexpr int NB = (FR_S + 1) * (K + 1) - 1;   // bucket ids [0, NB)
};

// LDS-resident cut of the key space.
struct FrTab {
  uint64_t spl[FR_S];        // sorted sample keys, KEY_SENTINEL-padded
  double lo[FR_S + 1];       // interval lower bound (value)
  double inv[FR_S + 1];      // K / (hi - lo), or 0 when the width is 0 / not finite
};

__device__ __forceinline__ uint64_t shfl_up1_u64(uint64_t v) {
  const int lo = __shfl_up((int)(uint32_t)v, 1);
  const int hi = __shfl_up((int)(uint32_t)(v >> 32), 1);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// Ascending bitonic sort of one key per lane across a wave (lane l ends with the l-th
// smallest); no LDS, no barrier.
__device__ __forceinline__ uint64_t wave_sort64(uint64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const uint64_t o = shfl_xor_u64(v, j);
      const bool up = (lane & k) == 0;
      const bool lower = (lane & j) == 0;
      const uint64_t lo = v < o ? v : o, hi = v < o ? o : v;
      v = (lower == up) ? lo : hi;
    }
  }
  return v;
}

__device__ __forceinline__ double fr_inv(double lo, double hi, double kf) {
  const double w = hi - lo;
  double inv = (w > 0.0 && w < INFINITY) ? kf / w : 0.0;
  return (inv < INFINITY) ? inv : 0.0;
}

// Wave 0 only: sort the sample keys (one per lane) and fill the interval table.
// vmin / vmax bound every key that will be bucketed (a superset's bounds are fine).
template <int K>
__device__ void fr_build_w0(FrTab& T, uint64_t sample_key, double vmin, double vmax) {
  const int lane = threadIdx.x & 63;
  const uint64_t s = wave_sort64(sample_key);
  const uint64_t prev = shfl_up1_u64(s);
  const int ns = __popcll(__ballot(s != KEY_SENTINEL));
  T.spl[lane] = s;
  const double kf = (double)K;
  double lo = 0.0, inv = 0.0;
  if (lane <= ns) {
    lo = lane == 0 ? vmin : okey_inv(prev);
    const double hi = lane == ns ? vmax : okey_inv(s);
    inv = fr_inv(lo, hi, kf);
  }
  T.lo[lane] = lo;
  T.inv[lane] = inv;
  if (lane == 63) {                       // interval 64 exists only when ns == 64
    double lo64 = 0.0, inv64 = 0.0;
    if (ns == 64) {
      lo64 = okey_inv(s);
      inv64 = fr_inv(lo64, vmax, kf);
    }
    T.lo[64] = lo64;
    T.inv[64] = inv64;
  }
}

// Bucket id of a (non-sentinel) key with value v = okey_inv(key).
template <int K>
__device__ __forceinline__ int fr_bucket(const FrTab& T, uint64_t key, double v) {
  int i = 0;
#pragma unroll
  for (int step = 32; step >= 1; step >>= 1)
    if (T.spl[i + step - 1] <= key) i += step;
  const uint64_t last = T.spl[i];
  i += last <= key;                         // i = #samples <= key, in [0, 64]
  if (i > 0 && T.spl[i - 1] == key) return (i - 1) * (K + 1) + K;
  const double inv = T.inv[i];
  const double t = (v - T.lo[i]) * inv;
  const int sub = inv > 0.0 ? (int)fmin(t, (double)(K - 1)) : 0;
  return i * (K + 1) + sub;
}

// Positional sample of lane l: the element at the middle of the l-th of 64 equal strides
// (NaN / absent -> sentinel).
__device__ __forceinline__ uint64_t fr_sample(const double* x, const uint8_t* prow, int64_t A) {
  const int lane = threadIdx.x & 63;
  const int64_t pos = ((int64_t)lane * A) / FR_S + A / (2 * FR_S);
  uint64_t sk = KEY_SENTINEL;
  if (pos < A && (prow ? prow[pos] != 0 : true)) {
    const double v = x[pos];
    if (v == v) sk = okey(v);
  }
  return sk;
}

// In-place exclusive scan of c[0..n) with c[n] = total, by a block of NT threads (each
// owns a run of SC consecutive entries).  Every thread must call it.  scr: NT/64 Ts.
template <int NT, class T>
__device__ void fr_scan(T* c, int n, T* scr) {
  constexpr int NW = NT / 64;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int sc = (n + 1 + NT - 1) / NT;
  const int b0 = t * sc;
  T loc = 0;
  for (int j = 0; j < sc; ++j)
    if (b0 + j < n) loc += c[b0 + j];
  T incl = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T u = __shfl_up(incl, o);
    if (lane >= o) incl += u;
  }
  if (lane == 63) scr[wid] = incl;
  __syncthreads();
  T base = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) base += (w < wid) ? scr[w] : (T)0;
  base += incl - loc;
  for (int j = 0; j < sc; ++j) {
    const int b = b0 + j;
    if (b < n) {
      const T x = c[b];
      c[b] = base;
      base += x;
    } else if (b == n) {
      c[b] = base;
    }
  }
  __syncthreads();
}

}  // namespace fmx
