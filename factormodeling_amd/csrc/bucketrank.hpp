// Splitter-bucket ranking of one row (fp64 keys) by a 256-thread workgroup.
//
// The exact average rank of x among the members of a row is
//     rank = #{y < x} + (#{y == x} + 1) / 2.
// Instead of sorting the row (the reference sorts: pandas rank_1d / scipy rankdata),
// a regular sample of NT keys is sorted and deduplicated into U <= NT splitters that cut
// the key space into 2U+1 buckets: "strictly between two splitters" (even ids) and
// "equal to splitter k" (odd ids).  Bucket ids are monotone in the key, so
//     #{y < x} = (members in lower buckets) + (members of x's bucket that are < x)
// and the in-bucket count needs a scan of only the ~A/NT keys of x's own bucket (none
// at all for equal-to-splitter buckets, which absorb heavy ties).  Counts are kept per
// membership mask (bit m of a member byte) so one bucketing serves several subsets,
// e.g. the pair-valid sets of the lag-1 and lag-2 ICs.
//
// Elements live in registers: thread t owns row positions t + k*NT, k < EMAX.
#pragma once

#include "rowkit.hpp"

namespace fmx {

template <int NT>
struct BRShared {
  static constexpr int NB = 2 * NT + 1;
  uint64_t spl[NT];        // sorted sample, then the U distinct splitters
  uint64_t tmp[NT];        // per-wave sorted sample lists
  int cnt[3][NB];          // members per bucket, per mask
  int start[3][NB];        // exclusive prefix of cnt
  int cursor[NB];
  int iscr[NT / 64 + 4];
  double dscr[16 * (NT / 64)];
  int U;
};

template <int NT>
__device__ __forceinline__ int bucket_of(const BRShared<NT>& S, uint64_t key) {
  int lo = 0, hi = S.U;
  while (lo < hi) {
    int m = (lo + hi) >> 1;
    if (S.spl[m] < key) lo = m + 1; else hi = m;
  }
  return (lo < S.U && S.spl[lo] == key) ? 2 * lo + 1 : 2 * lo;
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m);
  const int hi = __shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

__device__ __forceinline__ int lb64(const uint64_t* L, int n, uint64_t k) {
  int lo = 0, hi = n;
  while (lo < hi) { int m = (lo + hi) >> 1; if (L[m] < k) lo = m + 1; else hi = m; }
  return lo;
}
__device__ __forceinline__ int ub64(const uint64_t* L, int n, uint64_t k) {
  int lo = 0, hi = n;
  while (lo < hi) { int m = (lo + hi) >> 1; if (L[m] <= k) lo = m + 1; else hi = m; }
  return lo;
}

// Sort the NT sampled keys (one per thread, KEY_SENTINEL = no sample) and keep the
// distinct non-sentinel ones in S.spl[0..U).  Each wave sorts its 64 keys with an
// xor-shuffle bitonic network (no barriers); a key's final position is its index in its
// own wave plus the number of keys of the other waves that precede it (upper_bound in
// lower-numbered waves, lower_bound in higher ones), i.e. a stable NT/64-way merge.
template <int NT>
__device__ void br_splitters(BRShared<NT>& S, uint64_t mykey) {
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
  S.tmp[t] = v;
  __syncthreads();
  int pos = lane;
  for (int w = 0; w < NT / 64; ++w) {
    if (w == wid) continue;
    pos += (w < wid) ? ub64(S.tmp + w * 64, 64, v) : lb64(S.tmp + w * 64, 64, v);
  }
  S.spl[pos] = v;
  __syncthreads();
  const uint64_t u = S.spl[t];
  const int flag = (u != KEY_SENTINEL) && (t == 0 || S.spl[t - 1] != u);
  int U;
  const int p = block_exscan<NT>(flag, S.iscr, &U);
  if (flag) S.tmp[p] = u;
  __syncthreads();
  if (t < U) S.spl[t] = S.tmp[t];
  if (t == 0) S.U = U;
  __syncthreads();
}

// Bucketed member arrays (LDS): bkey[slot] key, binfo[slot] = bucket | mask << 10,
// bidx[slot] = position of the element in the row.
constexpr int BR_MSHIFT = 10;

// One element's per-mask in-bucket counts (keys strictly less / equal among members of
// mask m).  Callers iterate slots in bucket order so that the lanes of a wave share
// buckets: the scan loop lengths agree and the LDS reads broadcast.
template <int NT>
__device__ __forceinline__ void br_inbucket(const BRShared<NT>& S, const uint64_t* bkey, const uint16_t* binfo,
                                            int b, uint64_t key, int nmask, int* lt, int* eq) {
  for (int m = 0; m < nmask; ++m) { lt[m] = 0; eq[m] = 0; }
  if (b & 1) {
    for (int m = 0; m < nmask; ++m) eq[m] = S.cnt[m][b];
    return;
  }
  const int s0 = S.start[0][b], e0 = s0 + S.cnt[0][b];
  for (int q = s0; q < e0; ++q) {
    const uint64_t y = bkey[q];
    const int mm = binfo[q] >> BR_MSHIFT;
    const bool l = y < key, e = y == key;
    for (int m = 0; m < nmask; ++m) {
      const bool in = (mm >> m) & 1;
      lt[m] += in && l;
      eq[m] += in && e;
    }
  }
}

// Exclusive scans of the per-bucket counts of every mask.
template <int NT>
__device__ void br_scan(BRShared<NT>& S, int nmask) {
  constexpr int NB = BRShared<NT>::NB;
  constexpr int C = (NB + NT - 1) / NT;
  for (int m = 0; m < nmask; ++m) {
    const int b0 = threadIdx.x * C;
    int loc = 0;
    for (int c = 0; c < C; ++c) if (b0 + c < NB) loc += S.cnt[m][b0 + c];
    int tot;
    int base = block_exscan<NT>(loc, S.iscr, &tot);
    for (int c = 0; c < C; ++c)
      if (b0 + c < NB) { S.start[m][b0 + c] = base; base += S.cnt[m][b0 + c]; }
  }
  __syncthreads();
}

// Sum N doubles across the block with one LDS round trip; results in v[].
template <int NT, int N>
__device__ void block_sum_vec(double* v, double* scr) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i)
    for (int o = 32; o > 0; o >>= 1) v[i] += __shfl_xor(v[i], o);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < N; ++i) scr[wid * N + i] = v[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double t = 0.0;
    for (int w = 0; w < NT / 64; ++w) t += scr[w * N + i];
    v[i] = t;
  }
  __syncthreads();
}

// Order statistic k (0-based) among members of mask 0, using the bucket structure.
// Every thread gets the key.  Uses S.iscr[...] as a broadcast slot.
template <int NT, int EMAX>
__device__ uint64_t br_select(BRShared<NT>& S, const uint64_t* bkey, int k, uint64_t* bcast) {
  constexpr int NB = BRShared<NT>::NB;
  // bucket containing rank k: last b with start <= k and cnt > 0
  if (threadIdx.x == 0) {
    int lo = 0, hi = NB - 1;
    while (lo < hi) {
      int m = (lo + hi + 1) >> 1;
      if (S.start[0][m] <= k) lo = m; else hi = m - 1;
    }
    while (lo > 0 && S.cnt[0][lo] == 0) --lo;
    S.iscr[NT / 64] = lo;
  }
  __syncthreads();
  const int b = S.iscr[NT / 64];
  const int s0 = S.start[0][b], n = S.cnt[0][b];
  if (b & 1) {
    if (threadIdx.x == 0) *bcast = S.spl[b >> 1];
  } else {
    const int r = k - s0;
    for (int q = threadIdx.x; q < n; q += NT) {
      const uint64_t y = bkey[s0 + q];
      int lt = 0, eq = 0;
      for (int z = 0; z < n; ++z) {
        const uint64_t w = bkey[s0 + z];
        lt += w < y;
        eq += w == y;
      }
      if (lt <= r && r < lt + eq) *bcast = y;   // all writers store the same key
    }
  }
  __syncthreads();
  const uint64_t out = *bcast;
  __syncthreads();
  return out;
}

}  // namespace fmx
