// Block-level building blocks for per-row (cross-sectional) kernels.
//
// * block_pw_sum: numpy's float64 pairwise summation (add.reduce), bit-for-bit, driven by
//   a host-built schedule for the row length n (see pw_schedule in capi.hip).  pandas'
//   nanmean/nanvar (Series.mean()/.std()) sum with it, so reproducing its tree makes the
//   cross-sectional moments bit-identical to the reference.
// * block_exscan: exclusive prefix sum of one int per thread.
// * bitonic sort of (uint64 key, uint16 idx) pairs in LDS, ordered by (key, idx) so that
//   ties come out in position order (pandas method='first' / stable ordering).
#pragma once

#include "fmx_common.hpp"

namespace fmx {

// Schedule blob layout (int32):
//   [0] n  [1] L (#leaves, 0 => n < 8: sequential from 0)  [2] I (#internal nodes)
//   [3] R (#combine rounds)  [4] root node id
//   [5 .. 5+L)            leaf start
//   [5+L .. 5+2L)         leaf length
//   [5+2L .. 5+2L+R+1)    round offsets into the triple list
//   [.. + 3I)             (dst, left, right) node triples, grouped by round
struct PwView {
  const int32_t* b;
  __device__ int n() const { return b[0]; }
  __device__ int L() const { return b[1]; }
  __device__ int I() const { return b[2]; }
  __device__ int R() const { return b[3]; }
  __device__ int root() const { return b[4]; }
  __device__ int lstart(int k) const { return b[5 + k]; }
  __device__ int llen(int k) const { return b[5 + L() + k]; }
  __device__ int roff(int r) const { return b[5 + 2 * L() + r]; }
  __device__ const int32_t* trip() const { return b + 5 + 2 * L() + R() + 1; }
};

// nodes: LDS scratch of >= 2L doubles (+1).  Returns the sum to every thread.
template <int NT, class Elem>
__device__ double block_pw_sum(Elem elem, const int32_t* __restrict__ sched, double* nodes) {
  PwView s{sched};
  const int L = s.L();
  const int tid = threadIdx.x;
  if (L == 0) {
    if (tid == 0) {
      double r = 0.0;
      const int n = s.n();
      for (int i = 0; i < n; ++i) r += elem(i);
      nodes[0] = r;
    }
    __syncthreads();
    double r = nodes[0];
    __syncthreads();
    return r;
  }
  for (int t0 = 0; t0 < L * 8; t0 += NT) {
    const int t = t0 + tid;
    const bool act = t < L * 8;
    const int leaf = t >> 3, j = t & 7;
    double r = 0.0;
    int st = 0, len = 0, stop = 0;
    if (act) {
      st = s.lstart(leaf);
      len = s.llen(leaf);
      stop = len - (len & 7);
      r = elem(st + j);
      for (int i = 8; i < stop; i += 8) r += elem(st + i + j);
    }
    // ((r0+r1)+(r2+r3)) + ((r4+r5)+(r6+r7)) as an xor butterfly (IEEE + commutes)
    r = r + __shfl_xor(r, 1);
    r = r + __shfl_xor(r, 2);
    r = r + __shfl_xor(r, 4);
    if (act && j == 0) {
      for (int i = stop; i < len; ++i) r += elem(st + i);
      nodes[leaf] = r;
    }
  }
  __syncthreads();
  const int R = s.R();
  const int32_t* tr = s.trip();
  for (int rr = 0; rr < R; ++rr) {
    for (int q = s.roff(rr) + tid; q < s.roff(rr + 1); q += NT) {
      nodes[tr[3 * q]] = nodes[tr[3 * q + 1]] + nodes[tr[3 * q + 2]];
    }
    __syncthreads();
  }
  double r = nodes[s.root()];
  __syncthreads();
  return r;
}

// block_pw_sum with a barrier-light combine: all threads form the 8-lane leaves (and
// count the elements for which valid(i) holds), then wave 0 alone walks the combine
// rounds (in-order LDS within one wave: no block barrier per round) and publishes the
// root.  Returns the sum; *count receives the number of valid elements.
// nodes: >= 2L+1 doubles; iscr: >= NT/64 + 1 ints.
// side(): run by wave 1 while wave 0 combines (independent work that would otherwise take
// a serial phase of its own; it must not touch nodes / iscr).
struct PwNoSide {
  __device__ void operator()() const {}
};
template <int NT, class Elem, class Valid, class Side = PwNoSide>
__device__ double block_pw_sum_w0(Elem elem, Valid valid, const int32_t* __restrict__ sched, double* nodes,
                                  int* iscr, int* count, Side side = Side()) {
  PwView s{sched};
  const int L = s.L(), n = s.n();
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int c = 0;
  if (L == 0) {
    for (int i = tid; i < n; i += NT) c += valid(i);
  } else {
    for (int t0 = 0; t0 < L * 8; t0 += NT) {
      const int t = t0 + tid;
      const bool act = t < L * 8;
      const int leaf = t >> 3, j = t & 7;
      double r = 0.0;
      int st = 0, len = 0, stop = 0;
      if (act) {                       // numpy leaves hold >= 8 elements
        st = s.lstart(leaf);
        len = s.llen(leaf);
        stop = len - (len & 7);
        r = elem(st + j);
        c += valid(st + j);
        for (int i = 8; i < stop; i += 8) { r += elem(st + i + j); c += valid(st + i + j); }
      }
      // ((r0+r1)+(r2+r3)) + ((r4+r5)+(r6+r7)) as an xor butterfly (IEEE + commutes)
      r = r + __shfl_xor(r, 1);
      r = r + __shfl_xor(r, 2);
      r = r + __shfl_xor(r, 4);
      if (act && j == 0) {
        for (int i = stop; i < len; ++i) { r += elem(st + i); c += valid(st + i); }
        nodes[leaf] = r;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if (lane == 0) iscr[wid] = c;
  __syncthreads();
  if (wid == 0) {
    if (L == 0) {
      if (lane == 0) {
        double r = 0.0;
        for (int i = 0; i < n; ++i) r += elem(i);
        nodes[0] = r;
      }
    } else {
      const int R = s.R();
      const int32_t* tr = s.trip();
      for (int rr = 0; rr < R; ++rr) {
        for (int q = s.roff(rr) + lane; q < s.roff(rr + 1); q += 64)
          nodes[tr[3 * q]] = nodes[tr[3 * q + 1]] + nodes[tr[3 * q + 2]];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // round r visible to round r+1
      }
      if (lane == 0) nodes[0] = nodes[s.root()];
    }
    if (lane == 0) {
      int tot = 0;
      for (int w = 0; w < NT / 64; ++w) tot += iscr[w];
      iscr[NT / 64] = tot;
    }
  } else if (wid == 1) {
    side();
  }
  __syncthreads();
  const double r = nodes[0];
  *count = iscr[NT / 64];
  __syncthreads();
  return r;
}

// block_pw_sum for a row whose numpy pairwise tree is COMPLETE over NT/8 = 64 leaves (every
// leaf at depth 6: pw_tree64(n) on the host, e.g. n = 5000), with no serial combine phase.
// Thread t forms lane t & 7 of leaf t >> 3 as block_pw_sum_w0 does (the leaf's tail by its
// lane 0, then broadcast to the 8 lanes); the tree's first three levels pair adjacent leaves,
// i.e. lanes t ^ 8, t ^ 16, t ^ 32, so they are xor shuffles inside the wave (IEEE + commutes:
// a node's value does not depend on which child is added first); the wave's subtree sum goes
// to wsum[wid] and every thread adds the 8 wave sums in the tree's order after one barrier.
// side(): run by wave 1 before the barrier (as in block_pw_sum_w0).  wsum: 8 doubles per call
// site (a second call needs its own, or a barrier in between).
template <int NT, class Elem, class Side = PwNoSide>
__device__ double block_pw_sum_t64(Elem elem, const int32_t* __restrict__ sched, double* wsum, Side side = Side()) {
  static_assert(NT == 512, "64 leaves x 8 lanes");
  PwView s{sched};
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int leaf = tid >> 3, j = tid & 7;
  const int st = s.lstart(leaf), len = s.llen(leaf), stop = len - (len & 7);
  double r = elem(st + j);
  for (int i = 8; i < stop; i += 8) r += elem(st + i + j);
  r = r + __shfl_xor(r, 1);
  r = r + __shfl_xor(r, 2);
  r = r + __shfl_xor(r, 4);
  if (j == 0)
    for (int i = stop; i < len; ++i) r += elem(st + i);
  r = __shfl(r, lane & ~7);                   // the leaf's total (with its tail) to all 8 lanes
  r = r + __shfl_xor(r, 8);
  r = r + __shfl_xor(r, 16);
  r = r + __shfl_xor(r, 32);
  if (lane == 0) wsum[wid] = r;
  if (wid == 1) side();
  __syncthreads();
  return ((wsum[0] + wsum[1]) + (wsum[2] + wsum[3])) + ((wsum[4] + wsum[5]) + (wsum[6] + wsum[7]));
}

// Exclusive scan of v across the block; *total receives the sum.  scratch: NT/64 ints.
template <int NT>
__device__ int block_exscan(int v, int* scratch, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    int u = __shfl_up(incl, o);
    if (lane >= o) incl += u;
  }
  if (lane == 63) scratch[wid] = incl;
  __syncthreads();
  int base = 0, tot = 0;
  for (int w = 0; w < NT / 64; ++w) {
    int x = scratch[w];
    if (w < wid) base += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return base + incl - v;
}

template <int NT>
__device__ double block_sum(double v, double* scratch) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  double t = 0.0;
  for (int w = 0; w < NT / 64; ++w) t += scratch[w];
  __syncthreads();
  return t;
}

template <int NT>
__device__ double block_max(double v, double* scratch) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  double t = scratch[0];
  for (int w = 1; w < NT / 64; ++w) t = fmax(t, scratch[w]);
  __syncthreads();
  return t;
}

template <int NT>
__device__ double block_min(double v, double* scratch) {
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  double t = scratch[0];
  for (int w = 1; w < NT / 64; ++w) t = fmin(t, scratch[w]);
  __syncthreads();
  return t;
}

__device__ __forceinline__ bool kv_greater(uint64_t ka, uint32_t ia, uint64_t kb, uint32_t ib) {
  return ka > kb || (ka == kb && ia > ib);
}

// Bitonic sort of P (power of two) (key, idx) pairs in LDS, ascending by (key, idx).
template <int NT>
__device__ void bitonic_sort(uint64_t* key, uint16_t* idx, int P) {
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < (P >> 1); t += NT) {
        const int i = 2 * t - (t & (j - 1));
        const int l = i + j;
        const bool up = (i & k) == 0;
        uint64_t a = key[i], b = key[l];
        uint16_t ia = idx[i], ib = idx[l];
        bool gt = kv_greater(a, ia, b, ib);
        if (gt == up) {
          key[i] = b; key[l] = a;
          idx[i] = ib; idx[l] = ia;
        }
      }
      __syncthreads();
    }
  }
}

// Bitonic sort with a 16-bit group as the primary key: (grp, key, idx).
template <int NT>
__device__ void bitonic_sort_grp(uint64_t* key, uint16_t* idx, uint16_t* grp, int P) {
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < (P >> 1); t += NT) {
        const int i = 2 * t - (t & (j - 1));
        const int l = i + j;
        const bool up = (i & k) == 0;
        uint64_t a = key[i], b = key[l];
        uint16_t ia = idx[i], ib = idx[l], ga = grp[i], gb = grp[l];
        bool gt = ga > gb || (ga == gb && kv_greater(a, ia, b, ib));
        if (gt == up) {
          key[i] = b; key[l] = a;
          idx[i] = ib; idx[l] = ia;
          grp[i] = gb; grp[l] = ga;
        }
      }
      __syncthreads();
    }
  }
}

// first index p in [lo, hi) with key[p] >= k  /  > k
__device__ __forceinline__ int lower_bound_u64(const uint64_t* key, int lo, int hi, uint64_t k) {
  while (lo < hi) {
    int m = (lo + hi) >> 1;
    if (key[m] < k) lo = m + 1; else hi = m;
  }
  return lo;
}
__device__ __forceinline__ int upper_bound_u64(const uint64_t* key, int lo, int hi, uint64_t k) {
  while (lo < hi) {
    int m = (lo + hi) >> 1;
    if (key[m] <= k) lo = m + 1; else hi = m;
  }
  return lo;
}

// numpy percentile(method='linear') on the first n ascending sorted keys at fraction q.
__device__ __forceinline__ double sorted_percentile(const uint64_t* key, int n, double q) {
  double vi = (double)(n - 1) * q;
  double a, b, g;
  if (vi >= (double)(n - 1)) {
    a = b = okey_inv(key[n - 1]);
    g = vi + 1.0;
  } else {
    double pf = floor(vi);
    int p = (int)pf;
    g = vi - pf;
    a = okey_inv(key[p]);
    b = okey_inv(key[p + 1]);
  }
  double diff = b - a;
  return (g >= 0.5) ? b - diff * (1.0 - g) : a + diff * g;
}

inline int next_pow2(int n) {
  int p = 1;
  while (p < n) p <<= 1;
  return p;
}

// Device view of the cached schedules for every row length n <= nmax.
struct PwTable {
  const int32_t* off;   // [nmax + 1]
  const int32_t* blob;
  __device__ const int32_t* get(int n) const { return blob + off[n]; }
};
// Host: schedule table covering every n <= nmax on the current device (capi.hip).
PwTable pw_table(int nmax, fmx_status* err);
// Host: length in ints of the schedule blob for n.
int pw_len(int n);
// Host: numpy's pairwise tree for n is complete over 64 leaves (block_pw_sum_t64 applies).
bool pw_tree64(int n);
// Schedules up to this many ints are staged in LDS by the dense-row moment kernels.
constexpr int PW_LDS_MAX = 1024;

// Host: bucket-rank launchers (rank_ops.hip).
fmx_status br_cs_rank(const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld, int method,
                      const uint8_t* present, hipStream_t st);
fmx_status br_cs_rank_winsor(const double* X, double* Yr, double* Yw, int64_t F, int64_t D, int64_t A, int64_t ld,
                             double qlo, double qhi, const uint8_t* present, fmx_rank2_t* RK, hipStream_t st);
bool gram_zc_fits(int64_t A);
fmx_status gram_zc_pass(const double* X, int64_t F, int64_t D, int64_t A, int64_t ld, int64_t dc0, int64_t ndc,
                        double* Zc, int64_t apad, uint32_t* bits, int64_t nd_all, int64_t nwd, void* stream);
fmx_status br_cs_rank_winsor_zn(const double* X, double* Yr, double* Yw, double* Yz, double* Yn, int64_t F, int64_t D,
                                int64_t A, int64_t ld, int64_t d0, int64_t d1, double qlo, double qhi,
                                fmx_rank2_t* RK, PwTable pw, int slen, hipStream_t st);
fmx_status br_cs_rank2(const double* X, fmx_rank2_t* RK, int64_t F, int64_t D, int64_t A, int64_t ld, int64_t d0,
                       int64_t d1, hipStream_t st);
fmx_status br_cs_quantile(int op, const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                          double qlo, double qhi, const uint8_t* present, hipStream_t st);
fmx_status br_ic_daily(const double* X, const double* R, int64_t F, int64_t D, int64_t A, int64_t ld,
                       const int32_t* lags_host, int n_lags, double* out, hipStream_t st);
fmx_status br_ic_ranked(const double* X, const fmx_rank2_t* RK, const double* R, int64_t F, int64_t D, int64_t A,
                        int64_t ld, const int32_t* lags_host, int n_lags, double* out, int32_t* work, hipStream_t st);
int64_t ic_ranked_work_len(int64_t F, int64_t D);
fmx_status br_cs_rank_winsor_ic(const double* X, double* Yr, double* Yw, const double* R, int64_t F, int64_t D,
                                int64_t A, int64_t ld, double qlo, double qhi, const int32_t* lags, int n_lags,
                                fmx_rank2_t* RK, int32_t* work, double* out, hipStream_t st);
int64_t rank_ic_work_len(int64_t F, int64_t D, int64_t A);

}  // namespace fmx
