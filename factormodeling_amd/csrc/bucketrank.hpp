// Splitter-bucket ranking of one row (fp64 keys) by one workgroup.
//
// The exact average rank of x among the members of a row is
//     rank = #{y < x} + (#{y == x} + 1) / 2.
// The reference sorts (pandas rank_1d / scipy rankdata).  Here a regular positional
// sample of NS = NT keys is sorted (duplicates kept) into the splitter array spl[0..NS)
// that cuts the key space into NB = 2*NS+1 buckets: "strictly between spl[i-1] and
// spl[i]" (even id 2i) and "equal to spl[i]" (odd id 2i+1).  Bucket ids are monotone in
// the key, so
//     #{y < x} = (members of lower buckets) + (members of x's bucket that are < x)
// and the in-bucket count needs a scan of only the ~A/NS keys of x's own bucket (none at
// all for equal-to-splitter buckets, which absorb heavy ties).
//
// Elements live in registers (thread t owns row positions t + k*NT, k < EMAX).  A row
// costs one global read, ~8 barriers and 8 B of LDS per element (the bucketed keys), so
// three workgroups fit a CU at A = 5000 and the output is written coalesced by the
// owning thread.
#pragma once

#include "rowkit.hpp"

namespace fmx {

// Geometry of a row workgroup of NT threads (512 or 1024): NS = NT splitter samples (one
// per thread), NB = 2*NS+1 buckets, NW waves, SC scan entries per thread.
template <int NT>
struct BRG {
  static constexpr int NS = NT;
  static constexpr int NB = 2 * NS + 1;
  static constexpr int NW = NT / 64;
  static constexpr int SC = (NB + 1 + NT - 1) / NT;
};

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m);
  const int hi = __shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

// #{L[i] < k} (le = false) or #{L[i] <= k} (le = true) over a sorted 64-entry list:
// fixed-depth and branch-free, so the searches of one thread overlap their LDS reads.
__device__ __forceinline__ int count64(const uint64_t* L, uint64_t k, bool le) {
  int lo = 0;
#pragma unroll
  for (int step = 32; step >= 1; step >>= 1) {
    const uint64_t y = L[lo + step - 1];
    if (y < k || (le && y == k)) lo += step;
  }
  const uint64_t y = L[lo];                  // lo <= 63
  return lo + (y < k || (le && y == k));
}

// Sorts the NT sampled keys (one per thread; KEY_SENTINEL = no sample, sorts last) into
// spl[0..NT).  Each wave sorts its 64 keys with an xor-shuffle bitonic network (no
// barriers); a key's final position is its index in its own wave plus the number of keys
// of the other waves that precede it (upper_bound in lower-numbered waves, lower_bound in
// higher ones), i.e. a stable NT/64-way merge.  tmp: NT uint64 of LDS scratch.
template <int NT>
__device__ void br_splitters(uint64_t* spl, uint64_t* tmp, uint64_t mykey) {
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  uint64_t v = mykey;
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
  tmp[t] = v;
  __syncthreads();
  int pos = lane;
#pragma unroll
  for (int w = 0; w < BRG<NT>::NW; ++w) {
    // stable merge: equal keys of lower waves precede, of higher waves follow
    const int c = count64(tmp + w * 64, v, w < wid);
    pos += (w == wid) ? 0 : c;
  }
  spl[pos] = v;
  __syncthreads();
}

// Bucket id of a (non-sentinel) key: branch-free lower_bound over the NS splitters.
template <int NT>
__device__ __forceinline__ int br_bucket(const uint64_t* spl, uint64_t key) {
  constexpr int NS = BRG<NT>::NS;
  int lo = 0;
#pragma unroll
  for (int step = NS / 2; step >= 1; step >>= 1)
    if (spl[lo + step - 1] < key) lo += step;
  lo += spl[lo] < key;                       // lo == NS when every splitter is < key
  return (lo < NS && spl[lo] == key) ? 2 * lo + 1 : 2 * lo;
}

// In-place exclusive scan of c[0..NB) with c[NB] = total, for NV interleaved arrays
// (c + v*stride).  Every thread must call it.  scr: NV*NW ints.
template <int NT, int NV>
__device__ void br_scan(int* c, int stride, int* scr) {
  constexpr int BR_NB = BRG<NT>::NB, BR_NW = BRG<NT>::NW, BR_SC = BRG<NT>::SC;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int b0 = t * BR_SC;
  int loc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    loc[v] = 0;
#pragma unroll
    for (int j = 0; j < BR_SC; ++j)
      if (b0 + j < BR_NB) loc[v] += c[v * stride + b0 + j];
  }
  int incl[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    incl[v] = loc[v];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(incl[v], o);
      if (lane >= o) incl[v] += u;
    }
    if (lane == 63) scr[v * BR_NW + wid] = incl[v];
  }
  __syncthreads();
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    int base = 0;
    for (int w = 0; w < wid; ++w) base += scr[v * BR_NW + w];
    base += incl[v] - loc[v];
#pragma unroll
    for (int j = 0; j < BR_SC; ++j) {
      const int b = b0 + j;
      if (b < BR_NB) {
        const int x = c[v * stride + b];
        c[v * stride + b] = base;
        base += x;
      } else if (b == BR_NB) {
        c[v * stride + b] = base;
      }
    }
  }
  __syncthreads();
}

// Sum N values of type T over the block (wave shuffles, then one LDS round in which
// thread i < N totals value i).  scr: (NW + 1) * N entries.
template <int NT, int N, class T>
__device__ void br_sum(T* v, T* scr) {
  constexpr int BR_NW = BRG<NT>::NW;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[i] += __shfl_xor(v[i], o);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < N; ++i) scr[wid * N + i] = v[i];
  }
  __syncthreads();
  if (t < N) {
    T s = scr[t];
#pragma unroll
    for (int w = 1; w < BR_NW; ++w) s += scr[w * N + t];
    scr[BR_NW * N + t] = s;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = scr[BR_NW * N + i];
  __syncthreads();
}

// Max of N doubles over the block.  scr: (NW + 1) * N doubles.
template <int NT, int N>
__device__ void br_max(double* v, double* scr) {
  constexpr int BR_NW = BRG<NT>::NW;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[i] = fmax(v[i], __shfl_xor(v[i], o));
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < N; ++i) scr[wid * N + i] = v[i];
  }
  __syncthreads();
  if (t < N) {
    double s = scr[t];
#pragma unroll
    for (int w = 1; w < BR_NW; ++w) s = fmax(s, scr[w * N + t]);
    scr[BR_NW * N + t] = s;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = scr[BR_NW * N + i];
  __syncthreads();
}

// Two-phase block reduction of several value groups in one LDS round: each group calls
// br_part (wave shuffle reduce; lane 0 stores its wave's partials at scr[wid*S + off]),
// then br_fin combines the NW partials of value i < S (sum for i < nsum, max otherwise)
// into scr[NW*S + i].  scr: (NW + 1) * S doubles.
template <int N, bool MAX>
__device__ __forceinline__ void br_part(const double* v, double* scr, int S, int off) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double x = v[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double y = __shfl_xor(x, o);
      x = MAX ? fmax(x, y) : x + y;
    }
    if (lane == 0) scr[wid * S + off + i] = x;
  }
}
template <int NT>
__device__ __forceinline__ void br_fin(double* scr, int S, int nsum) {
  constexpr int NW = BRG<NT>::NW;
  const int t = threadIdx.x;
  __syncthreads();
  if (t < S) {
    double x = scr[t];
    for (int w = 1; w < NW; ++w) x = (t < nsum) ? x + scr[w * S + t] : fmax(x, scr[w * S + t]);
    scr[NW * S + t] = x;
  }
  __syncthreads();
}

// Positional sample key for thread t: the element at t*A/NT (NaN/absent -> sentinel).
template <int NT>
__device__ __forceinline__ uint64_t br_sample(const double* x, const uint8_t* prow, int64_t A) {
  const int64_t pos = ((int64_t)threadIdx.x * A) / NT;
  uint64_t sk = KEY_SENTINEL;
  if (pos < A && (prow ? prow[pos] != 0 : true)) {
    const double v = x[pos];
    if (v == v) sk = okey(v);
  }
  return sk;
}

}  // namespace fmx
