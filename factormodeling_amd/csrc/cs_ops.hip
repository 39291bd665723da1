// Cross-sectional (per-date) kernels: one 256-thread workgroup per (factor, date) row of
// the [F][D][ld] panel.  The row (A contiguous fp64, asset-fastest) is staged in LDS
// once and reduced/sorted there.
//
// Reference: operations.py:54-86 (cs_rank, cs_winsor, cs_filter_center, cs_zscore,
// cs_bool, cs_mean), :88-101 (elementwise), :104-168 (bucket, group ops), :171-182
// (market_neutralize), :248-304 (cs_regression).
#include <vector>
#include <map>
#include <mutex>
#include <cstdlib>
#include "rowkit.hpp"

extern "C" int32_t fmx_debug_pw_schedule(int32_t n, int32_t* out, int32_t cap);

namespace fmx {

constexpr int CS_NT = 256;

// Stage the present values of row (f, d) into LDS v[0..n) in asset order and return n.
// Dense rows (present == nullptr) map v[i] = x[i].  pos (optional, u16) records the asset
// of each staged element for ragged rows.
__device__ int stage_row(const double* __restrict__ x, const uint8_t* __restrict__ prow, int64_t A,
                         double* v, uint16_t* pos, int* iscr) {
  if (!prow) {
    for (int64_t i = threadIdx.x; i < A; i += CS_NT) {
      v[i] = x[i];
      if (pos) pos[i] = (uint16_t)i;
    }
    __syncthreads();
    return (int)A;
  }
  const int64_t C = (A + CS_NT - 1) / CS_NT;
  const int64_t a0 = threadIdx.x * C, a1 = min<int64_t>(A, a0 + C);
  int cnt = 0;
  for (int64_t a = a0; a < a1; ++a) cnt += prow[a] != 0;
  int tot;
  int base = block_exscan<CS_NT>(cnt, iscr, &tot);
  for (int64_t a = a0; a < a1; ++a) {
    if (prow[a]) {
      v[base] = x[a];
      if (pos) pos[base] = (uint16_t)a;
      ++base;
    }
  }
  __syncthreads();
  return tot;
}

// stage_row for an NT-thread block (ragged rows only).
template <int NT>
__device__ int stage_row_nt(const double* __restrict__ x, const uint8_t* __restrict__ prow, int64_t A, double* v,
                            uint16_t* pos, int* iscr) {
  const int64_t C = (A + NT - 1) / NT;
  const int64_t a0 = threadIdx.x * C, a1 = min<int64_t>(A, a0 + C);
  int cnt = 0;
  for (int64_t a = a0; a < a1; ++a) cnt += prow[a] != 0;
  int tot;
  int base = block_exscan<NT>(cnt, iscr, &tot);
  for (int64_t a = a0; a < a1; ++a) {
    if (prow[a]) {
      v[base] = x[a];
      if (pos) pos[base] = (uint16_t)a;
      ++base;
    }
  }
  __syncthreads();
  return tot;
}

// ------------------------------------------------------------------------------------
// cs_zscore / cs_mean / market_neutralize (nanops.nanmean / nanvar(ddof=0), pairwise).
// 512 threads per row; the two numpy pairwise sums use block_pw_sum_w0 (wave 0 walks the
// combine rounds), so a row costs five block barriers.  Optional stats[row] = (mean, sd)
// (sd = sqrt(nanvar ddof=0); the builder's Gram z-score, oracle/gram.py); OP
// FMX_CS_STATS_ONLY writes only the stats.
constexpr int FMX_CS_STATS_ONLY = 3;
constexpr int CSM_NT = 512;

template <int OP>
__global__ void __launch_bounds__(CSM_NT)
k_cs_moment(const double* __restrict__ X, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld,
            const uint8_t* __restrict__ present, PwTable pw, double* __restrict__ stats, int slen,
            double* __restrict__ Y2) {
  extern __shared__ double lds[];
  __shared__ int32_t sch_l[PW_LDS_MAX];              // dense rows: the schedule for n = A
  const int64_t row = fmx_blk();                     // grid dim3(D, F)
  const int64_t d = row % D;
  const double* x = X + row * ld;
  double* y = Y ? Y + row * ld : nullptr;
  const uint8_t* prow = present ? present + d * ld : nullptr;
  double* v = lds;                                   // [A]
  uint16_t* pos = present ? (uint16_t*)(v + A) : nullptr;
  double* nodes = (double*)((char*)(v + A) + (present ? ((A * 2 + 15) & ~15) : 0));  // [2A/64+8]
  int* iscr = (int*)(nodes + (2 * (A / 64) + 8));
  int n;
  const bool sch_lds = !prow && slen <= PW_LDS_MAX;
  if (!prow) {
    // the schedule is staged with the row (same barrier): no global round trips inside
    // the serial combine rounds
    if (sch_lds) {
      const int32_t* g = pw.get((int)A);
      for (int i = threadIdx.x; i < slen; i += CSM_NT) sch_l[i] = g[i];
    }
    for (int64_t i = threadIdx.x; i < A; i += CSM_NT) v[i] = x[i];
    __syncthreads();
    n = (int)A;
  } else {
    n = stage_row_nt<CSM_NT>(x, prow, A, v, pos, iscr);
  }
  if (n == 0) {
    if (stats && threadIdx.x == 0) { stats[2 * row] = qnan(); stats[2 * row + 1] = qnan(); }
    return;
  }
  const int32_t* sch = sch_lds ? sch_l : pw.get(n);
  int cnt;
  const double s1 = block_pw_sum_w0<CSM_NT>([&](int i) { double t = v[i]; return t == t ? t : 0.0; },
                                            [&](int i) { return (int)(v[i] == v[i]); }, sch, nodes, iscr, &cnt);
  const double mean = cnt > 0 ? s1 / (double)cnt : qnan();
  double sd = 0.0;
  if (OP != FMX_CS_MEAN) {
    int c2;
    const double s2 = block_pw_sum_w0<CSM_NT>([&](int i) {
      double t = v[i];
      double z = t == t ? t : 0.0;
      double q = (mean - z) * (mean - z);
      return t == t ? q : 0.0;
    }, [](int) { return 0; }, sch, nodes, iscr, &c2);
    const double var = cnt > 0 ? s2 / (double)cnt : qnan();
    sd = sqrt(var);
  }
  if (stats && threadIdx.x == 0) { stats[2 * row] = mean; stats[2 * row + 1] = sd; }
  if (OP == FMX_CS_STATS_ONLY) return;
  const bool guard = (OP == FMX_CS_MARKET_NEUTRALIZE) && (sd == 0.0 || sd != sd);
  // Y2 (cs_zscore only): market_neutralize of the same row from the same moments
  double* y2 = (OP == FMX_CS_ZSCORE && Y2) ? Y2 + row * ld : nullptr;
  const bool guard2 = sd == 0.0 || sd != sd;
  for (int i = threadIdx.x; i < n; i += CSM_NT) {
    double t = v[i];
    double o;
    if (OP == FMX_CS_MEAN) o = mean;
    else if (guard) o = 0.0;
    else o = (t - mean) / sd;
    int64_t a = prow ? pos[i] : i;
    y[a] = o;
    if (y2) y2[a] = guard2 ? 0.0 : o;
  }
  if (prow) {
    for (int64_t a = threadIdx.x; a < A; a += CSM_NT)
      if (!prow[a]) { y[a] = qnan(); if (y2) y2[a] = qnan(); }
  }
}

// ------------------------------------------------------------------------------------
// Dense rows, register-resident variant of k_cs_moment (same numpy pairwise order, bit-
// identical).  Lane (leaf = tid / 8, j = tid % 8) loads exactly the elements its numpy
// accumulator adds -- leaf start + j + 8i -- straight from HBM into registers (8 lanes
// read 64 contiguous bytes), so the row is never staged in LDS: a workgroup holds only the
// schedule (staged once, the workgroup is persistent over rows) and the 2L leaf nodes,
// and occupancy is set by registers.  Requires L <= CSR_NT / 8 leaves of <= 128 elements.
constexpr int CSR_NT = 512;
constexpr int CSR_EL = 16;            // elements per lane: leaves hold <= 128 = 8 x 16

// v + (v of lane ^ 1, ^ 2, ^ 4): the 8-lane butterfly of a leaf's accumulators on DPP
// (quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror) -- no ds_bpermute address
// registers held across the row loop.  Each step adds a commutative pair, so every lane of
// the 8 holds the same ((r0+r1)+(r2+r3)) + ((r4+r5)+(r6+r7)) bits as the shuffle version.
template <int CTRL>
__device__ __forceinline__ double csr_dpp(double v) {
  const int2 u = __builtin_bit_cast(int2, v);
  int2 r;
  r.x = __builtin_amdgcn_update_dpp(0, u.x, CTRL, 0xf, 0xf, false);
  r.y = __builtin_amdgcn_update_dpp(0, u.y, CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, r);
}
__device__ __forceinline__ double csr_leaf_sum8(double r) {
  r = r + csr_dpp<0xB1>(r);     // quad_perm [1,0,3,2]: lane ^ 1
  r = r + csr_dpp<0x4E>(r);     // quad_perm [2,3,0,1]: lane ^ 2
  r = r + csr_dpp<0x141>(r);    // row_half_mirror: lane 7 - i, the other quad of the 8
  return r;
}
// FMX_CS_GRAM_Z (the wide Gram's z pass, fmx_gram_direct_exact): row r of a date chunk
// (factor r / nd, date d0 + r % nd of X) -> Zc row r (stride apad): z = (x - mean) / sd where
// x is valid and sd > 0, else 0, and zeros in the pad columns [A, apad); its validity bits
// (bit a of word a / 32) -> bits row (r / nd) * nd_all + r % nd.
constexpr int FMX_CS_GRAM_Z = 4;
struct CsrZc {
  double* Z;
  uint32_t* bits;
  int64_t nd, D, d0, apad, nd_all;
  int nwd;
};
constexpr int CSR_ZC_WORDS = 8 * CSR_EL * (CSR_NT / 8) / 32;   // bit words of the longest row

// NT: threads per workgroup (one row each); 256 for rows of <= 32 numpy leaves (the z pass)
template <int OP, int NT = CSR_NT>
__global__ void __launch_bounds__(NT, OP == FMX_CS_GRAM_Z ? 4 * NT / NT : 8)
k_cs_moment_rg(const double* __restrict__ X, double* __restrict__ Y, int64_t nrows, int64_t A, int64_t ld,
               PwTable pw, int slen, double* __restrict__ stats, double* __restrict__ Y2, int nts, CsrZc zc) {
  constexpr int ZCW = 8 * CSR_EL * (NT / 8) / 32;           // bit words of the longest row
  __shared__ int32_t sch[PW_LDS_MAX];
  __shared__ double nodes[2 * (NT / 8) + 8];
  __shared__ int iscr[NT / 64 + 2];
  __shared__ uint32_t bw[OP == FMX_CS_GRAM_Z ? ZCW : 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  {
    const int32_t* g = pw.get((int)A);
    for (int i = tid; i < slen; i += NT) sch[i] = g[i];
    if (OP == FMX_CS_GRAM_Z)
      for (int i = tid; i < ZCW; i += NT) bw[i] = 0u;
  }
  __syncthreads();
  PwView sv{sch};
  const int L = sv.L(), R = sv.R();
  const int leaf = tid >> 3, j = tid & 7;
  const bool act = leaf < L;
  const int32_t* tr = sv.trip();
  // combine rounds of wave 0 (the schedule's tree), result in nodes[0]
  auto combine = [&]() {
    if (wid == 0) {
      for (int rr = 0; rr < R; ++rr) {
        for (int q = sv.roff(rr) + lane; q < sv.roff(rr + 1); q += 64)
          nodes[tr[3 * q]] = nodes[tr[3 * q + 1]] + nodes[tr[3 * q + 2]];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      if (lane == 0) nodes[0] = nodes[sv.root()];
    }
  };
  for (int64_t row = blockIdx.x; row < nrows; row += gridDim.x) {
    // the leaf geometry is re-read from the LDS schedule per row (two LDS reads) rather
    // than held across the row loop, where it would spill
    const int st = act ? sv.lstart(leaf) : 0, len = act ? sv.llen(leaf) : 0;
    const int stop = len - (len & 7), nfull = stop >> 3;
    const double* x = X + (OP == FMX_CS_GRAM_Z ? ((row / zc.nd) * zc.D + zc.d0 + row % zc.nd) * ld : row * ld);
    double xv[CSR_EL];
#pragma unroll
    for (int i = 0; i < CSR_EL; ++i) xv[i] = (i < nfull) ? x[st + j + 8 * i] : 0.0;
    // sum 1: numpy nansum (NaN -> 0) and the valid count
    double r = 0.0;
    int c = 0;
#pragma unroll
    for (int i = 0; i < CSR_EL; ++i) {
      if (i < nfull) {
        const double t = xv[i];
        const double z = t == t ? t : 0.0;
        r = i == 0 ? z : r + z;
        c += t == t;
      }
    }
    r = csr_leaf_sum8(r);
    if (act && j == 0) {
      for (int q = stop; q < len; ++q) { const double t = x[st + q]; r += t == t ? t : 0.0; c += t == t; }
      nodes[leaf] = r;
    }
    // the wave's valid count from the bit planes of the lanes' counts (c < 32): ballots +
    // scalar popcounts, no cross-lane shuffles
    {
      int cw = 0;
#pragma unroll
      for (int b = 0; b < 5; ++b) cw += __popcll(__ballot((c >> b) & 1)) << b;
      c = cw;
    }
    if (lane == 0) iscr[wid] = c;
    __syncthreads();
    combine();
    if (tid == 0) {
      int tot = 0;
      for (int w = 0; w < NT / 64; ++w) tot += iscr[w];
      iscr[NT / 64] = tot;
    }
    __syncthreads();
    const int cnt = iscr[NT / 64];
    const double mean = cnt > 0 ? nodes[0] / (double)cnt : qnan();
    double sd = 0.0;
    if (OP != FMX_CS_MEAN) {
      __syncthreads();                                 // nodes[0] read by everyone
      double q2 = 0.0;
#pragma unroll
      for (int i = 0; i < CSR_EL; ++i) {
        if (i < nfull) {
          const double t = xv[i];
          const double z = t == t ? t : 0.0;
          const double q = t == t ? (mean - z) * (mean - z) : 0.0;
          q2 = i == 0 ? q : q2 + q;
        }
      }
      q2 = csr_leaf_sum8(q2);
      if (act && j == 0) {
        for (int q = stop; q < len; ++q) {
          const double t = x[st + q];
          const double z = t == t ? t : 0.0;
          q2 += t == t ? (mean - z) * (mean - z) : 0.0;
        }
        nodes[leaf] = q2;
      }
      __syncthreads();
      combine();
      __syncthreads();
      const double var = cnt > 0 ? nodes[0] / (double)cnt : qnan();
      sd = sqrt(var);
    }
    if (stats && tid == 0) { stats[2 * row] = cnt > 0 ? mean : qnan(); stats[2 * row + 1] = cnt > 0 ? sd : qnan(); }
    if (OP == FMX_CS_GRAM_Z) {
      const bool okr = sd > 0.0;                       // cnt > 0 and sigma not 0 (NaN fails)
      double* zr = zc.Z + row * zc.apad;
#pragma unroll
      for (int i = 0; i < CSR_EL; ++i)
        if (i < nfull) {
          const double t = xv[i];
          const bool ok = okr && t == t;
          zr[st + j + 8 * i] = ok ? (t - mean) / sd : 0.0;
          // the leaf's 8 lanes hold 8 consecutive assets: one byte of bits, OR-ed in by j == 0
          const uint32_t byte = (uint32_t)(__ballot(ok) >> (lane & 56)) & 0xffu;
          if (j == 0 && byte) {
            const int p = st + 8 * i, w = p >> 5, o = p & 31;
            atomicOr(&bw[w], byte << o);
            if (o > 24) atomicOr(&bw[w + 1], byte >> (32 - o));
          }
        }
      if (act && j == 0)
        for (int q = stop; q < len; ++q) {
          const double t = x[st + q];
          const bool ok = okr && t == t;
          zr[st + q] = ok ? (t - mean) / sd : 0.0;
          if (ok) atomicOr(&bw[(st + q) >> 5], 1u << ((st + q) & 31));
        }
      for (int64_t a = A + tid; a < zc.apad; a += NT) zr[a] = 0.0;
      __syncthreads();
      uint32_t* br = zc.bits + ((row / zc.nd) * zc.nd_all + row % zc.nd) * zc.nwd;
      for (int w = tid; w < zc.nwd; w += NT) {
        br[w] = bw[w];
        bw[w] = 0u;                                    // the next row's atomics follow the loop-end barrier
      }
    } else if (OP != FMX_CS_STATS_ONLY) {
      const bool guard = (OP == FMX_CS_MARKET_NEUTRALIZE) && (sd == 0.0 || sd != sd);
      auto outv = [&](double t) {
        if (OP == FMX_CS_MEAN) return mean;
        if (guard) return 0.0;
        return (t - mean) / sd;
      };
      double* y = Y + row * ld;
      auto put = [&](double v, double* p) {   // nts: write-once outputs as nontemporal stores
        if (nts) __builtin_nontemporal_store(v, p);
        else *p = v;
      };
      // market_neutralize of the same row from the same moments (sd in {0, NaN} -> 0),
      // stored next to each z so no output value stays live across a second loop
      const bool two = OP == FMX_CS_ZSCORE && Y2;
      const bool g2 = sd == 0.0 || sd != sd;
      double* y2 = two ? Y2 + row * ld : nullptr;
#pragma unroll
      for (int i = 0; i < CSR_EL; ++i)
        if (i < nfull) {
          const double o = outv(xv[i]);
          put(o, y + st + j + 8 * i);
          if (two) put(g2 ? 0.0 : o, y2 + st + j + 8 * i);
        }
      if (act && j == 0)
        for (int q = stop; q < len; ++q) {
          const double o = outv(x[st + q]);
          y[st + q] = o;
          if (two) y2[st + q] = g2 ? 0.0 : o;
        }
    }
    __syncthreads();                                   // nodes / iscr reused by the next row
  }
}

// ------------------------------------------------------------------------------------
// cs_rank: pandas Series.rank(method) over non-NaN, (r-1)/(len-1) with len = #rows of the
// date (NaN included), a single-row date -> 0.5.
__global__ void __launch_bounds__(CS_NT)
k_cs_rank(const double* __restrict__ X, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld,
          int P, int method, const uint8_t* __restrict__ present) {
  extern __shared__ uint64_t keys[];
  uint16_t* idx = (uint16_t*)(keys + P);
  int* iscr = (int*)(idx + P + 8);
  const int64_t d = blockIdx.x, f = blockIdx.y;
  const double* x = X + (f * D + d) * ld;
  double* y = Y + (f * D + d) * ld;
  const uint8_t* prow = present ? present + d * ld : nullptr;
  int nrow_l = 0, nv_l = 0;
  for (int i = threadIdx.x; i < P; i += CS_NT) {
    uint64_t k = KEY_SENTINEL;
    uint16_t id = 0xffff;
    if (i < A) {
      bool p = prow ? prow[i] != 0 : true;
      if (p) {
        double t = x[i];
        nrow_l += 1;
        if (t == t) { k = okey(t); id = (uint16_t)i; nv_l += 1; }
      }
    }
    keys[i] = k;
    idx[i] = id;
  }
  int nrow, nv;
  block_exscan<CS_NT>(nrow_l, iscr, &nrow);
  block_exscan<CS_NT>(nv_l, iscr, &nv);
  if (method == FMX_RANK_AVERAGE_PROPAGATE && nv < nrow) {
    // scipy.stats.rankdata(nan_policy='propagate'): one NaN makes the whole row NaN
    for (int64_t a = threadIdx.x; a < A; a += CS_NT) y[a] = qnan();
    return;
  }
  const bool single_half = (method != FMX_RANK_AVERAGE_PROPAGATE) && nrow == 1;
  // NaN / absent rows are written here (sorted members are written below)
  for (int64_t a = threadIdx.x; a < A; a += CS_NT) {
    bool p = prow ? prow[a] != 0 : true;
    if (!p) y[a] = qnan();
    else if (!(x[a] == x[a])) y[a] = single_half ? 0.5 : qnan();
  }
  bitonic_sort<CS_NT>(keys, idx, P);
  // dense ranks need the number of distinct keys before each position
  int* dstart = nullptr;
  if (method == FMX_RANK_DENSE) {
    // chunked scan of group-start flags
    const int C = (nv + CS_NT - 1) / CS_NT;
    const int p0 = threadIdx.x * C, p1 = min(nv, p0 + C);
    int c = 0;
    for (int p = p0; p < p1; ++p) c += (p == 0 || keys[p] != keys[p - 1]);
    int tot;
    int base = block_exscan<CS_NT>(c, iscr, &tot);
    // store dense rank (1-based) of each position into the upper half of an int view of
    // the key array is not possible (keys still needed) -> recompute on the fly below
    dstart = iscr;  // unused marker
    for (int p = p0; p < p1; ++p) {
      base += (p == 0 || keys[p] != keys[p - 1]);
      double r = (double)base;
      int a = idx[p];
      y[a] = single_half ? 0.5 : (r - 1.0) / (double)(nrow - 1);
    }
    return;
  }
  (void)dstart;
  for (int p = threadIdx.x; p < nv; p += CS_NT) {
    uint64_t k = keys[p];
    int less = lower_bound_u64(keys, 0, p + 1, k);
    int eq = upper_bound_u64(keys, p, nv, k) - less;
    double r;
    switch (method) {
      case FMX_RANK_MIN: r = (double)(less + 1); break;
      case FMX_RANK_MAX: r = (double)(less + eq); break;
      case FMX_RANK_FIRST: r = (double)(p + 1); break;
      default: r = (double)less + (double)(eq + 1) / 2.0;
    }
    int a = idx[p];
    y[a] = single_half ? 0.5 : (r - 1.0) / (double)(nrow - 1);
  }
}

// ------------------------------------------------------------------------------------
// cs_winsor (OP 0) / cs_filter_center (OP 1): numpy linear percentiles of the non-NaN
// values (pandas Series.quantile -> np.percentile(q*100) / 100).
template <int OP>
__global__ void __launch_bounds__(CS_NT)
k_cs_quantile(const double* __restrict__ X, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld,
              int P, double qlo, double qhi, const uint8_t* __restrict__ present) {
  extern __shared__ uint64_t keys[];
  uint16_t* idx = (uint16_t*)(keys + P);
  int* iscr = (int*)(idx + P + 8);
  double* qv = (double*)(iscr + 16);
  const int64_t d = blockIdx.x, f = blockIdx.y;
  const double* x = X + (f * D + d) * ld;
  double* y = Y + (f * D + d) * ld;
  const uint8_t* prow = present ? present + d * ld : nullptr;
  int nv_l = 0;
  for (int i = threadIdx.x; i < P; i += CS_NT) {
    uint64_t k = KEY_SENTINEL;
    if (i < A && (prow ? prow[i] != 0 : true)) {
      double t = x[i];
      if (t == t) { k = okey(t); nv_l += 1; }
    }
    keys[i] = k;
    idx[i] = (uint16_t)i;
  }
  int nv;
  block_exscan<CS_NT>(nv_l, iscr, &nv);
  bitonic_sort<CS_NT>(keys, idx, P);
  if (threadIdx.x == 0) {
    if (nv > 0) {
      qv[0] = sorted_percentile(keys, nv, qlo);
      qv[1] = sorted_percentile(keys, nv, qhi);
    } else {
      qv[0] = qv[1] = qnan();
    }
  }
  __syncthreads();
  const double lo = qv[0], hi = qv[1];
  for (int64_t a = threadIdx.x; a < A; a += CS_NT) {
    bool p = prow ? prow[a] != 0 : true;
    if (!p) { y[a] = qnan(); continue; }
    double t = x[a];
    double o;
    if (OP == 0) {
      o = t;
      if (nv >= 5) o = (t < lo) ? lo : ((t > hi) ? hi : t);
    } else {
      o = (t < lo || t > hi) ? t : 0.0;
    }
    y[a] = o;
  }
}

// ------------------------------------------------------------------------------------
// Group ops per (date, group): G[d][a] holds dense group ids (-1 = NaN group, dropped by
// the reference's groupby).  Elements are sorted by (group, key, asset); each group's
// members are then contiguous and in asset order for the pairwise sums.
template <int OP>
__global__ void __launch_bounds__(CS_NT)
k_group(const double* __restrict__ X, const int32_t* __restrict__ G, double* __restrict__ Y, int64_t D,
        int64_t A, int64_t ld, int P, int ngroups, int method, const uint8_t* __restrict__ present,
        PwTable pw) {
  extern __shared__ uint64_t keys[];
  uint16_t* idx = (uint16_t*)(keys + P);
  uint16_t* grp = idx + P;
  double* vals = (double*)(((uintptr_t)(grp + P) + 15) & ~(uintptr_t)15);  // [P] values in sorted order
  double* nodes = vals + P;                                              // [2P/64 + 8]
  int* iscr = (int*)(nodes + (2 * (P / 64) + 8));
  int* gbound = iscr + 16;                                               // [ngroups+1]
  const int64_t d = blockIdx.x, f = blockIdx.y;
  const double* x = X + (f * D + d) * ld;
  const int32_t* g = G + d * ld;
  double* y = Y + (f * D + d) * ld;
  const uint8_t* prow = present ? present + d * ld : nullptr;
  const bool by_value = (OP == 3);
  for (int i = threadIdx.x; i < P; i += CS_NT) {
    uint64_t k = KEY_SENTINEL;
    uint16_t gi = 0xffff;
    if (i < A && (prow ? prow[i] != 0 : true)) {
      int gg = g[i];
      if (gg >= 0) {
        gi = (uint16_t)gg;
        double t = x[i];
        k = by_value ? (t == t ? okey(t) : KEY_SENTINEL - 1) : 0;
      }
    }
    keys[i] = k;
    idx[i] = (uint16_t)i;
    grp[i] = gi;
  }
  // rows outside any group -> NaN
  for (int64_t a = threadIdx.x; a < A; a += CS_NT) {
    bool p = prow ? prow[a] != 0 : true;
    if (!p || g[a] < 0) y[a] = qnan();
  }
  bitonic_sort_grp<CS_NT>(keys, idx, grp, P);
  for (int i = threadIdx.x; i < P; i += CS_NT) vals[i] = (grp[i] != 0xffff) ? x[idx[i]] : 0.0;
  // group boundaries
  for (int gg = threadIdx.x; gg <= ngroups; gg += CS_NT) {
    int lo = 0, hi = P;
    while (lo < hi) { int m = (lo + hi) >> 1; if (grp[m] < gg) lo = m + 1; else hi = m; }
    gbound[gg] = lo;
  }
  __syncthreads();
  for (int gg = 0; gg < ngroups; ++gg) {
    const int s = gbound[gg], e = gbound[gg + 1], n = e - s;
    if (n == 0) continue;
    if (OP == 3) {
      // rank over non-NaN members (keys < SENTINEL-1); NaN members sort last in the group
      int nvl = 0;
      for (int p = s + threadIdx.x; p < e; p += CS_NT) nvl += keys[p] < KEY_SENTINEL - 1;
      int nvv;
      block_exscan<CS_NT>(nvl, iscr, &nvv);
      if (method == FMX_RANK_DENSE && nvv > 1) {
        // dense rank = #distinct keys <= k among the group's valid members (chunked scan)
        const int C = (nvv + CS_NT - 1) / CS_NT, p0 = s + threadIdx.x * C, p1 = min(s + nvv, p0 + C);
        int c = 0;
        for (int p = p0; p < p1; ++p) c += (p == s || keys[p] != keys[p - 1]);
        int tot;
        int base = block_exscan<CS_NT>(c, iscr, &tot);
        for (int p = p0; p < p1; ++p) {
          base += (p == s || keys[p] != keys[p - 1]);
          y[idx[p]] = ((double)base - 1.0) / (double)(nvv - 1);
        }
        for (int p = s + nvv + threadIdx.x; p < e; p += CS_NT) y[idx[p]] = qnan();
        continue;
      }
      for (int p = s + threadIdx.x; p < e; p += CS_NT) {
        int a = idx[p];
        if (nvv <= 1) { y[a] = 0.5; continue; }
        uint64_t k = keys[p];
        if (!(k < KEY_SENTINEL - 1)) { y[a] = qnan(); continue; }
        int less = lower_bound_u64(keys, s, p + 1, k) - s;
        int eq = upper_bound_u64(keys, p, s + nvv, k) - (less + s);
        double r;
        switch (method) {
          case FMX_RANK_MIN: r = (double)(less + 1); break;
          case FMX_RANK_MAX: r = (double)(less + eq); break;
          case FMX_RANK_FIRST: r = (double)(p - s + 1); break;
          default: r = (double)less + (double)(eq + 1) / 2.0;
        }
        y[a] = (r - 1.0) / (double)(nvv - 1);
      }
      continue;
    }
    const double* vg = vals + s;
    int cl = 0;
    for (int i = threadIdx.x; i < n; i += CS_NT) cl += vg[i] == vg[i];
    int cnt;
    block_exscan<CS_NT>(cl, iscr, &cnt);
    const int32_t* sch = pw.get(n);
    double s1 = block_pw_sum<CS_NT>([&](int i) { double t = vg[i]; return t == t ? t : 0.0; }, sch, nodes);
    double mean = cnt > 0 ? s1 / (double)cnt : qnan();
    double sd = 0.0;
    if (OP == 2) {
      double s2 = block_pw_sum<CS_NT>([&](int i) {
        double t = vg[i];
        double z = t == t ? t : 0.0;
        double q = (mean - z) * (mean - z);
        return t == t ? q : 0.0;
      }, sch, nodes);
      sd = sqrt(cnt > 0 ? s2 / (double)cnt : qnan());
    }
    const bool guard = (OP == 2) && (sd == 0.0 || sd != sd);
    for (int i = threadIdx.x; i < n; i += CS_NT) {
      double t = vg[i];
      double o;
      if (OP == 0) o = mean;
      else if (OP == 1) o = t - mean;
      else o = guard ? 0.0 : (t - mean) / sd;
      y[idx[s + i]] = o;
    }
  }
}

// ------------------------------------------------------------------------------------
// cs_regression: per date OLS on pair-valid rows (population moments, pandas means).
__global__ void __launch_bounds__(CS_NT)
k_cs_regression(const double* __restrict__ Yv, const double* __restrict__ Xv, double* __restrict__ Out,
                int64_t D, int64_t A, int64_t ld, int rettype, const uint8_t* __restrict__ present,
                PwTable pw) {
  extern __shared__ double lds[];
  double* xs = lds;            // [A]
  double* ys = xs + A;         // [A]
  uint16_t* pos = (uint16_t*)(ys + A);
  double* nodes = (double*)((char*)pos + ((A * 2 + 15) & ~15));
  int* iscr = (int*)(nodes + (2 * (A / 64) + 8));
  const int64_t d = blockIdx.x;
  const double* x = Xv + d * ld;
  const double* yv = Yv + d * ld;
  double* o = Out + d * ld;
  const uint8_t* prow = present ? present + d * ld : nullptr;
  // compact pair-valid rows in asset order
  const int64_t C = (A + CS_NT - 1) / CS_NT;
  const int64_t a0 = threadIdx.x * C, a1 = min<int64_t>(A, a0 + C);
  int cnt = 0;
  for (int64_t a = a0; a < a1; ++a) {
    bool ok = (prow ? prow[a] != 0 : true) && x[a] == x[a] && yv[a] == yv[a];
    cnt += ok;
  }
  int n;
  int base = block_exscan<CS_NT>(cnt, iscr, &n);
  for (int64_t a = a0; a < a1; ++a) {
    bool ok = (prow ? prow[a] != 0 : true) && x[a] == x[a] && yv[a] == yv[a];
    if (ok) { xs[base] = x[a]; ys[base] = yv[a]; pos[base] = (uint16_t)a; ++base; }
    o[a] = qnan();
  }
  __syncthreads();
  if (n < 2) return;
  const int32_t* sch = pw.get(n);
  const double dn = (double)n;
  double mx = block_pw_sum<CS_NT>([&](int i) { return xs[i]; }, sch, nodes) / dn;
  double my = block_pw_sum<CS_NT>([&](int i) { return ys[i]; }, sch, nodes) / dn;
  double cov = block_pw_sum<CS_NT>([&](int i) { return (xs[i] - mx) * (ys[i] - my); }, sch, nodes) / dn;
  double var_x = block_pw_sum<CS_NT>([&](int i) { double t = xs[i] - mx; return t * t; }, sch, nodes) / dn;
  double beta = cov / var_x;
  double alpha = my - beta * mx;
  double r2 = 0.0;
  if (rettype == 4) {
    double var_y = block_pw_sum<CS_NT>([&](int i) { double t = ys[i] - my; return t * t; }, sch, nodes) / dn;
    r2 = (cov * cov) / (var_x * var_y);
  }
  for (int i = threadIdx.x; i < n; i += CS_NT) {
    double fitted = alpha + beta * xs[i];
    double r;
    switch (rettype) {
      case 0: r = ys[i] - fitted; break;   // resid
      case 1: r = beta; break;
      case 2: r = alpha; break;
      case 3: r = fitted; break;
      default: r = r2;
    }
    o[pos[i]] = r;
  }
}

// ------------------------------------------------------------------------------------
// Elementwise (operations.py:80-101) and bucket codes (pd.cut, :104-110).
__global__ void k_elementwise(const double* __restrict__ X, double* __restrict__ Y, int64_t n, int op,
                              double a, double b) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    double v = X[i], o;
    switch (op) {
      case FMX_EW_SIGN: o = (v > 0) ? 1.0 : ((v < 0) ? -1.0 : (v == v ? 0.0 : v)); break;  // np.sign(-0.) = +0.
      case FMX_EW_POWER:
        // ndarray.__pow__ fast paths (numpy fast_scalar_power), reached via Series.__pow__
        if (a == 2.0) o = v * v;
        else if (a == 0.5) o = sqrt(v);
        else if (a == 1.0) o = v;
        else if (a == -1.0) o = 1.0 / v;
        else if (a == 0.0) o = 1.0;
        else o = pow(v, a);
        break;
      case FMX_EW_LOG: o = log(v); break;
      case FMX_EW_ABS: o = fabs(v); break;
      case FMX_EW_CLIP: o = (v < a) ? a : ((v > b) ? b : v); break;
      case FMX_EW_WHERE: o = (v != 0.0) ? a : b; break;   // cond as 0/1 (NaN -> true)
      default: o = v;
    }
    Y[i] = o;
  }
}

__global__ void k_bucket(const double* __restrict__ X, int32_t* __restrict__ codes, int64_t n,
                         const double* __restrict__ edges, int ne) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    double v = X[i];
    int c = -1;
    if (v == v) {
      // searchsorted(edges, v, side='left')
      int lo = 0, hi = ne;
      while (lo < hi) { int m = (lo + hi) >> 1; if (edges[m] < v) lo = m + 1; else hi = m; }
      int id = (v == edges[0]) ? 1 : lo;
      if (id > 0 && id <= ne - 1) c = id - 1;
    }
    codes[i] = c;
  }
}

static fmx_status set_lds(const void* k, size_t lds) {
  if (lds > 160 * 1024) {
    set_error("row too long for the LDS-resident cross-sectional kernels (" + std::to_string(lds) + " B)");
    return FMX_ERR_UNSUPPORTED;
  }
  if (lds > 64 * 1024) FMX_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  return FMX_OK;
}

}  // namespace fmx

using namespace fmx;

static fmx_status cs_moment_launch(int op, const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                                   const uint8_t* present, double* stats, void* stream, double* Y2 = nullptr) {
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  fmx_status e = FMX_OK;
  PwTable pw = pw_table((int)A, &e);
  if (e) return e;
  size_t lds = A * 8 + (present ? ((A * 2 + 15) & ~15) : 0) + (2 * (A / 64) + 8) * 8 + 16 * 4 + 64;
  const void* k = op == FMX_CS_ZSCORE ? (const void*)k_cs_moment<FMX_CS_ZSCORE>
                : op == FMX_CS_MEAN ? (const void*)k_cs_moment<FMX_CS_MEAN>
                : op == FMX_CS_MARKET_NEUTRALIZE ? (const void*)k_cs_moment<FMX_CS_MARKET_NEUTRALIZE>
                                                 : (const void*)k_cs_moment<FMX_CS_STATS_ONLY>;
  if ((e = set_lds(k, lds))) return e;
  FMX_ARG(F * D <= 0x7fffffffll, "too many rows");
  int slen = present ? PW_LDS_MAX + 1 : pw_len((int)A);
  // dense rows whose numpy leaves fit one 512-thread workgroup: register-resident kernel
  static const bool no_rg = getenv("FMX_CS_MOMENT_LDS") != nullptr;
  if (!present && slen <= PW_LDS_MAX && !no_rg && A >= 8) {
    std::vector<int32_t> sh(slen);
    fmx_debug_pw_schedule((int32_t)A, sh.data(), slen);
    bool fits = sh[1] > 0 && sh[1] <= CSR_NT / 8;
    for (int k = 0; fits && k < sh[1]; ++k) fits = sh[5 + sh[1] + k] <= 8 * CSR_EL;
    if (fits) {
      const void* kr = op == FMX_CS_ZSCORE ? (const void*)k_cs_moment_rg<FMX_CS_ZSCORE>
                     : op == FMX_CS_MEAN ? (const void*)k_cs_moment_rg<FMX_CS_MEAN>
                     : op == FMX_CS_MARKET_NEUTRALIZE ? (const void*)k_cs_moment_rg<FMX_CS_MARKET_NEUTRALIZE>
                                                      : (const void*)k_cs_moment_rg<FMX_CS_STATS_ONLY>;
      static std::map<const void*, int64_t> slots_cache;
      static std::mutex mu;
      int64_t slots;
      {
        std::lock_guard<std::mutex> g(mu);
        auto it = slots_cache.find(kr);
        if (it == slots_cache.end()) {
          int dev = 0, cus = 0, per = 0;
          FMX_HIP(hipGetDevice(&dev));
          FMX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
          FMX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kr, CSR_NT, 0));
          it = slots_cache.emplace(kr, (int64_t)std::max(1, per) * std::max(1, cus)).first;
        }
        slots = it->second;
      }
      const int64_t nrows = F * D;
      const int64_t grid = std::min<int64_t>(nrows, slots);
      static const int nts = getenv("FMX_CS_NT") ? atoi(getenv("FMX_CS_NT")) : 0;   // A/B: nontemporal stores
      CsrZc zc{};
      void* rargs[] = {(void*)&X, (void*)&Y, (void*)&nrows, (void*)&A, (void*)&ld, (void*)&pw, (void*)&slen,
                       (void*)&stats, (void*)&Y2, (void*)&nts, (void*)&zc};
      FMX_HIP(hipLaunchKernel(kr, dim3((unsigned)grid), dim3(CSR_NT), rargs, 0, as_stream(stream)));
      return FMX_OK;
    }
  }
  void* args[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&present, (void*)&pw, (void*)&stats,
                  (void*)&slen, (void*)&Y2};
  FMX_HIP(hipLaunchKernel(k, fmx_grid2(D, F), dim3(CSM_NT), args, lds, as_stream(stream)));
  return FMX_OK;
}

extern "C" fmx_status fmx_cs_moment(int32_t op, const double* X, double* Y, int64_t F, int64_t D, int64_t A,
                                    int64_t ld, const uint8_t* present, void* stream) {
  FMX_ARG(X && Y, "null panel");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  FMX_ARG(op >= FMX_CS_ZSCORE && op <= FMX_CS_MARKET_NEUTRALIZE, "unknown cs op");
  return cs_moment_launch(op, X, Y, F, D, A, ld, present, nullptr, stream);
}

// The wide Gram's z pass (FMX_CS_GRAM_Z above) over dates [dc0, dc0 + ndc) of X [F][D][ld]:
// the row stats in numpy's pairwise order (as fmx_cs_moment_stats), Zc [F][ndc][apad] and the
// validity bits [F][nd_all][nwd] (rows of this chunk).  FMX_ERR_UNSUPPORTED when the row does
// not fit the register-resident kernel (the caller keeps the stats + tile-kernel z path).
namespace fmx {
// leaves of the numpy schedule of n = A (0: does not fit the register-resident kernel)
static int gram_zc_leaves(int64_t A) {
  if (A < 8 || ceil_div(A, (int64_t)32) > CSR_ZC_WORDS) return 0;
  const int slen = pw_len((int)A);
  if (slen > PW_LDS_MAX) return 0;
  std::vector<int32_t> sh(slen);
  fmx_debug_pw_schedule((int32_t)A, sh.data(), slen);
  bool fits = sh[1] > 0 && sh[1] <= CSR_NT / 8;
  for (int k = 0; fits && k < sh[1]; ++k) fits = sh[5 + sh[1] + k] <= 8 * CSR_EL;
  return fits ? sh[1] : 0;
}
bool gram_zc_fits(int64_t A) { return gram_zc_leaves(A) > 0; }

fmx_status gram_zc_pass(const double* X, int64_t F, int64_t D, int64_t A, int64_t ld, int64_t dc0, int64_t ndc,
                        double* Zc, int64_t apad, uint32_t* bits, int64_t nd_all, int64_t nwd, void* stream) {
  if (F == 0 || ndc == 0 || A == 0) return FMX_OK;
  if (!gram_zc_fits(A) || nwd != ceil_div(A, (int64_t)32) || apad < A) return FMX_ERR_UNSUPPORTED;
  fmx_status e = FMX_OK;
  PwTable pw = pw_table((int)A, &e);
  if (e) return e;
  int slen = pw_len((int)A);
  // rows of <= 32 leaves (A <= ~4096): 256-thread workgroups, every lane holding a leaf's
  // elements, twice the rows in flight per CU (FMX_GRAM_ZC_NT=512: the A/B arm)
  static const int want = [] { const char* e = getenv("FMX_GRAM_ZC_NT"); return e ? atoi(e) : 256; }();
  const bool half = want == 256 && gram_zc_leaves(A) <= 32;
  const int nt = half ? 256 : CSR_NT;
  const void* kr = half ? (const void*)k_cs_moment_rg<FMX_CS_GRAM_Z, 256> : (const void*)k_cs_moment_rg<FMX_CS_GRAM_Z>;
  static int64_t slots_cache[2] = {0, 0};
  int64_t& slots = slots_cache[half ? 1 : 0];
  if (!slots) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kr, nt, 0) != hipSuccess)
      slots = 256;
    else
      slots = (int64_t)std::max(1, per) * std::max(1, cus);
  }
  const int64_t nrows = F * ndc;
  FMX_ARG(nrows <= 0x7fffffffll, "too many rows");
  const int64_t grid = std::min<int64_t>(nrows, slots);
  CsrZc zc{Zc, bits, ndc, D, dc0, apad, nd_all, (int)nwd};
  double *Y = nullptr, *stats = nullptr, *Y2 = nullptr;
  int nts = 0;
  void* rargs[] = {(void*)&X, (void*)&Y, (void*)&nrows, (void*)&A, (void*)&ld, (void*)&pw, (void*)&slen,
                   (void*)&stats, (void*)&Y2, (void*)&nts, (void*)&zc};
  FMX_HIP(hipLaunchKernel(kr, dim3((unsigned)grid), dim3(nt), rargs, 0, as_stream(stream)));
  return FMX_OK;
}
}  // namespace fmx

extern "C" fmx_status fmx_cs_moment_stats(int32_t op, const double* X, double* Y, int64_t F, int64_t D, int64_t A,
                                          int64_t ld, const uint8_t* present, double* stats, void* stream) {
  FMX_ARG(X && stats, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  FMX_ARG(op >= FMX_CS_ZSCORE && op <= FMX_CS_STATS, "unknown cs op");
  FMX_ARG(op == FMX_CS_STATS || Y, "null output panel");
  return cs_moment_launch(op, X, op == FMX_CS_STATS ? nullptr : Y, F, D, A, ld, present, stats, stream);
}

extern "C" fmx_status fmx_cs_zscore_neutralize(const double* X, double* Yz, double* Yn, int64_t F, int64_t D,
                                               int64_t A, int64_t ld, const uint8_t* present, double* stats,
                                               void* stream) {
  FMX_ARG(X && Yz && Yn, "null panel");
  FMX_ARG(Yz != X && Yn != X && Yz != Yn, "outputs must be distinct from X and each other");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  return cs_moment_launch(FMX_CS_ZSCORE, X, Yz, F, D, A, ld, present, stats, stream, Yn);
}

extern "C" fmx_status fmx_cs_rank(const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                                  int32_t method, const uint8_t* present, void* stream) {
  FMX_ARG(X && Y, "null panel");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  FMX_ARG(method >= FMX_RANK_AVERAGE && method <= FMX_RANK_AVERAGE_PROPAGATE, "unknown rank method");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  if (method != FMX_RANK_FIRST && method != FMX_RANK_DENSE)
    return br_cs_rank(X, Y, F, D, A, ld, method, present, as_stream(stream));
  int P = next_pow2((int)A);
  if (P < 2) P = 2;
  size_t lds = (size_t)P * 10 + 16 + 16 * 4 + 64;
  fmx_status e;
  if ((e = set_lds((const void*)k_cs_rank, lds))) return e;
  int m = method;
  void* args[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&P, (void*)&m, (void*)&present};
  FMX_HIP(hipLaunchKernel((const void*)k_cs_rank, dim3((unsigned)D, (unsigned)F), dim3(CS_NT), args, lds,
                          as_stream(stream)));
  return FMX_OK;
}

static fmx_status cs_quantile(int op, const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                              double qlo, double qhi, const uint8_t* present, void* stream) {
  FMX_ARG(X && Y, "null panel");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  if (A <= 16384) return br_cs_quantile(op, X, Y, F, D, A, ld, qlo, qhi, present, as_stream(stream));
  int P = next_pow2((int)A);
  if (P < 2) P = 2;
  size_t lds = (size_t)P * 10 + 16 + 16 * 4 + 16 + 64;
  const void* k = op == 0 ? (const void*)k_cs_quantile<0> : (const void*)k_cs_quantile<1>;
  fmx_status e;
  if ((e = set_lds(k, lds))) return e;
  void* args[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&P, (void*)&qlo, (void*)&qhi,
                  (void*)&present};
  FMX_HIP(hipLaunchKernel(k, dim3((unsigned)D, (unsigned)F), dim3(CS_NT), args, lds, as_stream(stream)));
  return FMX_OK;
}

extern "C" fmx_status fmx_cs_winsor(const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                                    double qlo, double qhi, const uint8_t* present, void* stream) {
  return cs_quantile(0, X, Y, F, D, A, ld, qlo, qhi, present, stream);
}

extern "C" fmx_status fmx_cs_rank_winsor(const double* X, double* Yrank, double* Ywinsor, int64_t F, int64_t D,
                                         int64_t A, int64_t ld, double qlo, double qhi, const uint8_t* present,
                                         fmx_rank2_t* rank2, void* stream) {
  FMX_ARG(X && Yrank && Ywinsor, "null panel");
  FMX_ARG(Yrank != X && Ywinsor != X && Yrank != Ywinsor, "outputs must be distinct from X and each other");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  FMX_ARG(!(rank2 && present), "rank2 ranks every non-NaN cell: no presence mask");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  fmx_status e = br_cs_rank_winsor(X, Yrank, Ywinsor, F, D, A, ld, qlo, qhi, present, rank2, as_stream(stream));
  if (e != FMX_ERR_UNSUPPORTED) return e;
  // rows the fused kernel does not take (FMX_RANK_IMPL=br, or its LDS does not fit): the
  // doubled ranks from the ranks-only pass, then the two single-op passes
  if (rank2) {
    if (A > 16384) { set_error("rank2 needs the fused rank kernel (A <= 16384)"); return FMX_ERR_UNSUPPORTED; }
    if ((e = br_cs_rank2(X, rank2, F, D, A, ld, 0, D, as_stream(stream)))) return e;
  }
  if ((e = fmx_cs_rank(X, Yrank, F, D, A, ld, FMX_RANK_AVERAGE, present, stream))) return e;
  return cs_quantile(0, X, Ywinsor, F, D, A, ld, qlo, qhi, present, stream);
}

extern "C" fmx_status fmx_cs_rank_winsor_zn(const double* X, double* Yrank, double* Ywinsor, double* Yz, double* Yn,
                                            int64_t F, int64_t D, int64_t A, int64_t ld, double qlo, double qhi,
                                            fmx_rank2_t* rank2, void* stream) {
  FMX_ARG(X && Yrank && Ywinsor && Yz && Yn, "null panel");
  const double* outs[4] = {Yrank, Ywinsor, Yz, Yn};
  for (int i = 0; i < 4; ++i) {
    FMX_ARG(outs[i] != X, "outputs must be distinct from X");
    for (int j = i + 1; j < 4; ++j) FMX_ARG(outs[i] != outs[j], "outputs must be distinct from each other");
  }
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  fmx_status e = FMX_OK;
  PwTable pw = pw_table((int)A, &e);
  if (e) return e;
  e = br_cs_rank_winsor_zn(X, Yrank, Ywinsor, Yz, Yn, F, D, A, ld, 0, D, qlo, qhi, rank2, pw, pw_len((int)A),
                           as_stream(stream));
  if (e != FMX_ERR_UNSUPPORTED) return e;
  // rows the fused kernel does not take: rank + winsor, then the moments
  if ((e = fmx_cs_rank_winsor(X, Yrank, Ywinsor, F, D, A, ld, qlo, qhi, nullptr, rank2, stream))) return e;
  return fmx_cs_zscore_neutralize(X, Yz, Yn, F, D, A, ld, nullptr, nullptr, stream);
}

extern "C" fmx_status fmx_cs_rank2(const double* X, fmx_rank2_t* rank2, int64_t F, int64_t D, int64_t A, int64_t ld,
                                   void* stream) {
  FMX_ARG(X && rank2, "null panel");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 16384, "bad dims (A <= 16384)");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  return br_cs_rank2(X, rank2, F, D, A, ld, 0, D, as_stream(stream));
}

// Date sub-ranges [d0, d1) of every factor of an [F][D][ld] panel (the sharded step: the
// owned dates before the halo exchange lands, the halo rows after it).  Fine-bucket rows only.
extern "C" fmx_status fmx_cs_rank_winsor_zn_dates(const double* X, double* Yrank, double* Ywinsor, double* Yz,
                                                  double* Yn, int64_t F, int64_t D, int64_t A, int64_t ld, int64_t d0,
                                                  int64_t d1, double qlo, double qhi, fmx_rank2_t* rank2,
                                                  void* stream) {
  FMX_ARG(X && Yrank && Ywinsor && Yz && Yn, "null panel");
  const double* outs[4] = {Yrank, Ywinsor, Yz, Yn};
  for (int i = 0; i < 4; ++i) {
    FMX_ARG(outs[i] != X, "outputs must be distinct from X");
    for (int j = i + 1; j < 4; ++j) FMX_ARG(outs[i] != outs[j], "outputs must be distinct from each other");
  }
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 16384, "bad dims (A <= 16384)");
  FMX_ARG(0 <= d0 && d0 <= d1 && d1 <= D, "date range outside the panel");
  if (F == 0 || d1 == d0 || A == 0) return FMX_OK;
  fmx_status e = FMX_OK;
  PwTable pw = pw_table((int)A, &e);
  if (e) return e;
  e = br_cs_rank_winsor_zn(X, Yrank, Ywinsor, Yz, Yn, F, D, A, ld, d0, d1, qlo, qhi, rank2, pw, pw_len((int)A),
                           as_stream(stream));
  if (e != FMX_ERR_UNSUPPORTED) return e;
  // rows the fused kernel does not take (FMX_RANK_IMPL=br, or its LDS does not fit): the
  // two-pass form of fmx_cs_rank_winsor_zn, one factor's date range [d0, d1) at a time (a
  // [1][d1 - d0][ld] panel at row (f, d0)) -- as the whole-panel entry falls back
  for (int64_t f = 0; f < F; ++f) {
    const int64_t o = (f * D + d0) * ld;
    fmx_rank2_t* rk = rank2 ? rank2 + o : nullptr;
    if ((e = fmx_cs_rank_winsor(X + o, Yrank + o, Ywinsor + o, 1, d1 - d0, A, ld, qlo, qhi, nullptr, rk, stream)))
      return e;
    if ((e = fmx_cs_zscore_neutralize(X + o, Yz + o, Yn + o, 1, d1 - d0, A, ld, nullptr, nullptr, stream))) return e;
  }
  return FMX_OK;
}

extern "C" fmx_status fmx_cs_rank2_dates(const double* X, fmx_rank2_t* rank2, int64_t F, int64_t D, int64_t A,
                                         int64_t ld, int64_t d0, int64_t d1, void* stream) {
  FMX_ARG(X && rank2, "null panel");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 16384, "bad dims (A <= 16384)");
  FMX_ARG(0 <= d0 && d0 <= d1 && d1 <= D, "date range outside the panel");
  if (F == 0 || d1 == d0 || A == 0) return FMX_OK;
  return br_cs_rank2(X, rank2, F, D, A, ld, d0, d1, as_stream(stream));
}

extern "C" fmx_status fmx_cs_filter_center(const double* X, double* Y, int64_t F, int64_t D, int64_t A,
                                           int64_t ld, double qlo, double qhi, const uint8_t* present,
                                           void* stream) {
  return cs_quantile(1, X, Y, F, D, A, ld, qlo, qhi, present, stream);
}

// ------------------------------------------------------------------------------------
// Group ops on long rows (k_group sorts the whole row in LDS: A <= 4096).  One 1024-thread
// workgroup per (date, factor) row keeps its cells in registers (cell t + k*GL_NT) and
// visits the groups one at a time: the group's members are compacted in asset order
// (ballot prefix per register chunk) into LDS and reduced with the numpy pairwise schedule
// of their count (the reference's x.mean() over the group's rows), then every owner
// writes its cells.  Rank: the group's (key, asset) pairs are bitonic-sorted in LDS and
// each owner binary-searches its key ('first': its (key, asset) pair; 'dense': the
// distinct-value prefix written over the sorted asset slots).
constexpr int GL_NT = 1024;
constexpr int GL_NW = GL_NT / 64;

template <int EMAX>
__device__ int gl_offsets(uint32_t flags, int* pre, int* wtot) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const uint64_t b = __ballot((flags >> k) & 1u);
    pre[k] = __popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0) wtot[k * GL_NW + wid] = __popcll(b);
  }
  __syncthreads();
  if (wid == 0) {
    constexpr int N = EMAX * GL_NW, PER = (N + 63) / 64;
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
  for (int k = 0; k < EMAX; ++k) pre[k] += wtot[k * GL_NW + wid];
  return wtot[EMAX * GL_NW];
}

template <int OP, int EMAX>
__global__ void __launch_bounds__(GL_NT)
k_group_long(const double* __restrict__ X, const int32_t* __restrict__ G, double* __restrict__ Y, int64_t D,
             int64_t A, int64_t ld, int ngroups, int method, const uint8_t* __restrict__ present, PwTable pw,
             int Pmax) {
  extern __shared__ uint64_t gl[];                // [Pmax] values / keys, then [Pmax] u16 asset slots
  __shared__ double nodes[2 * (16384 / 64) + 8];
  __shared__ int iscr[GL_NW + 2];
  __shared__ int wtot[EMAX * GL_NW + 1];
  const int t = threadIdx.x;
  const int64_t d = blockIdx.x, f = blockIdx.y;
  const double* x = X + (f * D + d) * ld;
  const int32_t* g = G + d * ld;
  double* y = Y + (f * D + d) * ld;
  const uint8_t* prow = present ? present + d * ld : nullptr;
  double xv[EMAX];
  int gv[EMAX];
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t a = t + (int64_t)k * GL_NT;
    const bool in = a < A && (!prow || prow[a]);
    xv[k] = a < A ? x[a] : 0.0;
    gv[k] = in ? g[a] : -1;
    if (a < A && gv[k] < 0) y[a] = qnan();       // absent row or NaN group
  }
  uint16_t* slot = (uint16_t*)(gl + Pmax);
  for (int gg = 0; gg < ngroups; ++gg) {
    uint32_t fl = 0;
#pragma unroll
    for (int k = 0; k < EMAX; ++k) fl |= (uint32_t)(gv[k] == gg) << k;
    int pre[EMAX];
    const int m = gl_offsets<EMAX>(fl, pre, wtot);
    if (m == 0) continue;                         // block-uniform
    if (OP != 3) {
      double* vals = reinterpret_cast<double*>(gl);
#pragma unroll
      for (int k = 0; k < EMAX; ++k)
        if ((fl >> k) & 1u) vals[pre[k]] = xv[k];
      __syncthreads();
      const int32_t* sch = pw.get(m);
      int cnt;
      const double s1 = block_pw_sum_w0<GL_NT>([&](int i) { const double v = vals[i]; return v == v ? v : 0.0; },
                                               [&](int i) { return (int)(vals[i] == vals[i]); }, sch, nodes, iscr,
                                               &cnt);
      const double mean = cnt > 0 ? s1 / (double)cnt : qnan();
      double sd = 0.0;
      if (OP == 2) {
        int c2;
        const double s2 = block_pw_sum_w0<GL_NT>([&](int i) {
          const double v = vals[i];
          const double z = v == v ? v : 0.0;
          const double q = (mean - z) * (mean - z);
          return v == v ? q : 0.0;
        }, [](int) { return 0; }, sch, nodes, iscr, &c2);
        sd = sqrt(cnt > 0 ? s2 / (double)cnt : qnan());
      }
      const bool guard = (OP == 2) && (sd == 0.0 || sd != sd);
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
        if (!((fl >> k) & 1u)) continue;
        const double v = xv[k];
        double o;
        if (OP == 0) o = mean;
        else if (OP == 1) o = v - mean;
        else o = guard ? 0.0 : (v - mean) / sd;
        y[t + (int64_t)k * GL_NT] = o;
      }
    } else {
      int P = 2;
      while (P < m) P <<= 1;
      if (P > Pmax) {                             // group larger than the sort buffer
#pragma unroll
        for (int k = 0; k < EMAX; ++k)
          if ((fl >> k) & 1u) y[t + (int64_t)k * GL_NT] = qnan();
        __syncthreads();
        continue;
      }
      uint64_t* keys = gl;
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
        if (!((fl >> k) & 1u)) continue;
        const double v = xv[k];
        keys[pre[k]] = v == v ? okey(v) : KEY_SENTINEL - 1;   // NaN members sort last
        slot[pre[k]] = (uint16_t)(t + k * GL_NT);
      }
      for (int i = m + t; i < P; i += GL_NT) { keys[i] = KEY_SENTINEL; slot[i] = 0xffff; }
      __syncthreads();
      bitonic_sort<GL_NT>(keys, slot, P);
      const int nvv = lower_bound_u64(keys, 0, m, KEY_SENTINEL - 1);
      if (method == FMX_RANK_DENSE && nvv > 1) {
        // dense rank of every sorted position, written over the (unused) asset slots
        const int C = (nvv + GL_NT - 1) / GL_NT, p0 = t * C, p1 = min(nvv, p0 + C);
        int c = 0;
        for (int p = p0; p < p1; ++p) c += (p == 0 || keys[p] != keys[p - 1]);
        int tot;
        int base = block_exscan<GL_NT>(c, iscr, &tot);
        for (int p = p0; p < p1; ++p) { base += (p == 0 || keys[p] != keys[p - 1]); slot[p] = (uint16_t)base; }
        __syncthreads();
      }
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
        if (!((fl >> k) & 1u)) continue;
        const double v = xv[k];
        const int64_t a = t + (int64_t)k * GL_NT;
        if (nvv <= 1) { y[a] = 0.5; continue; }
        if (!(v == v)) { y[a] = qnan(); continue; }
        const uint64_t kk = okey(v);
        const int less = lower_bound_u64(keys, 0, nvv, kk);
        const int eq = upper_bound_u64(keys, less, nvv, kk) - less;
        double r;
        if (method == FMX_RANK_MIN) r = (double)(less + 1);
        else if (method == FMX_RANK_MAX) r = (double)(less + eq);
        else if (method == FMX_RANK_DENSE) r = (double)slot[less];
        else if (method == FMX_RANK_FIRST) {
          int lo = less, hi = less + eq;              // ties sorted by asset
          while (lo < hi) { const int md = (lo + hi) >> 1; if (slot[md] < (uint16_t)a) lo = md + 1; else hi = md; }
          r = (double)(lo + 1);
        } else r = (double)less + (double)(eq + 1) / 2.0;
        y[a] = (r - 1.0) / (double)(nvv - 1);
      }
    }
    __syncthreads();                              // LDS reused by the next group
  }
}

// Group mean / neutralize / normalize on rows past 16,384 assets (operations.py:112-149),
// where k_group_long's register-resident row and LDS compaction end.  The row stays in HBM
// (L2-resident while its workgroup walks it); per group the members are compacted in asset
// order into the workgroup's slice of a global scratch (block scan per 1024-cell chunk) and
// reduced with the numpy pairwise schedule of their count -- the same arithmetic, in the
// same order, as k_group_long, so the outputs are bit-identical to it.  Persistent
// workgroups (gridDim.x of them, A doubles of scratch each) walk the (factor, date) rows.
// Codes outside [0, ngroups) and absent cells belong to no group (NaN).
template <int OP>
__global__ void __launch_bounds__(GL_NT)
k_group_xl(const double* __restrict__ X, const int32_t* __restrict__ G, double* __restrict__ Y, int64_t F, int64_t D,
           int64_t A, int64_t ld, int ngroups, const uint8_t* __restrict__ present, PwTable pw,
           double* __restrict__ scratch) {
  __shared__ double nodes[2 * (65536 / 64) + 8];
  __shared__ int iscr[GL_NW + 2];
  const int t = threadIdx.x;
  double* vals = scratch + (int64_t)blockIdx.x * A;
  for (int64_t row = blockIdx.x; row < F * D; row += gridDim.x) {
    const int64_t f = row / D, d = row % D;
    const double* x = X + (f * D + d) * ld;
    const int32_t* g = G + d * ld;
    double* y = Y + (f * D + d) * ld;
    const uint8_t* prow = present ? present + d * ld : nullptr;
    auto code = [&](int64_t a) {
      const int c = (!prow || prow[a]) ? g[a] : -1;
      return (c >= 0 && c < ngroups) ? c : -1;
    };
    for (int64_t a = t; a < A; a += GL_NT)
      if (code(a) < 0) y[a] = qnan();
    for (int gg = 0; gg < ngroups; ++gg) {
      int m = 0;
      for (int64_t c0 = 0; c0 < A; c0 += GL_NT) {
        const int64_t a = c0 + t;
        const bool mem = a < A && code(a) == gg;
        int tot;
        const int off = block_exscan<GL_NT>(mem ? 1 : 0, iscr, &tot);
        if (mem) vals[m + off] = x[a];
        m += tot;
        __syncthreads();                          // iscr reused by the next chunk's scan
      }
      if (m == 0) continue;                       // block-uniform
      const int32_t* sch = pw.get(m);
      int cnt;
      const double s1 = block_pw_sum_w0<GL_NT>([&](int i) { const double v = vals[i]; return v == v ? v : 0.0; },
                                               [&](int i) { return (int)(vals[i] == vals[i]); }, sch, nodes, iscr,
                                               &cnt);
      const double mean = cnt > 0 ? s1 / (double)cnt : qnan();
      double sd = 0.0;
      if (OP == 2) {
        int c2;
        const double s2 = block_pw_sum_w0<GL_NT>([&](int i) {
          const double v = vals[i];
          const double z = v == v ? v : 0.0;
          const double q = (mean - z) * (mean - z);
          return v == v ? q : 0.0;
        }, [](int) { return 0; }, sch, nodes, iscr, &c2);
        sd = sqrt(cnt > 0 ? s2 / (double)cnt : qnan());
      }
      const bool guard = (OP == 2) && (sd == 0.0 || sd != sd);
      for (int64_t a = t; a < A; a += GL_NT) {
        if (code(a) != gg) continue;
        const double v = x[a];
        double o;
        if (OP == 0) o = mean;
        else if (OP == 1) o = v - mean;
        else o = guard ? 0.0 : (v - mean) / sd;
        y[a] = o;
      }
      __syncthreads();                            // scratch reused by the next group
    }
  }
}

static int64_t group_xl_grid(int64_t rows) {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return std::max(n, 1);
  }();
  return std::max<int64_t>(1, std::min<int64_t>(rows, 2 * (int64_t)cus));
}

extern "C" int64_t fmx_group_op_long_work_bytes(int64_t F, int64_t D, int64_t A) {
  if (F <= 0 || D <= 0 || A <= 0) return 0;
  return (int64_t)sizeof(double) * group_xl_grid(F * D) * A;
}

extern "C" fmx_status fmx_group_op_long(int32_t op, const double* X, const int32_t* G, double* Y, int64_t F, int64_t D,
                                        int64_t A, int64_t ld, int32_t ngroups, const uint8_t* present, void* work,
                                        int64_t work_bytes, void* stream) {
  FMX_ARG(X && G && Y && Y != X, "null / aliased panel");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  FMX_ARG(op >= FMX_GROUP_MEAN && op <= FMX_GROUP_NORMALIZE, "group mean / neutralize / normalize (rank: "
                                                               "fmx_group_rank_sorted)");
  FMX_ARG(ngroups >= 0, "bad group count");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  if (!work || work_bytes < fmx_group_op_long_work_bytes(F, D, A)) {
    set_error("workspace smaller than fmx_group_op_long_work_bytes()");
    return FMX_ERR_ARG;
  }
  fmx_status e = FMX_OK;
  PwTable pw = pw_table((int)A, &e);
  if (e) return e;
  const void* k = op == FMX_GROUP_MEAN ? (const void*)k_group_xl<0>
                : op == FMX_GROUP_NEUTRALIZE ? (const void*)k_group_xl<1> : (const void*)k_group_xl<2>;
  int ng = ngroups;
  double* scr = static_cast<double*>(work);
  void* args[] = {(void*)&X, (void*)&G, (void*)&Y, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&ng,
                  (void*)&present, (void*)&pw, (void*)&scr};
  FMX_HIP(hipLaunchKernel(k, dim3((unsigned)group_xl_grid(F * D)), dim3(GL_NT), args, 0, as_stream(stream)));
  return FMX_OK;
}

extern "C" fmx_status fmx_group_op(int32_t op, const double* X, const int32_t* G, double* Y, int64_t F,
                                   int64_t D, int64_t A, int64_t ld, int32_t ngroups, int32_t method,
                                   const uint8_t* present, void* stream) {
  FMX_ARG(X && G && Y, "null panel");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  FMX_ARG(op >= FMX_GROUP_MEAN && op <= FMX_GROUP_RANK, "unknown group op");
  FMX_ARG(ngroups >= 0 && ngroups < 65535, "bad group count");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  fmx_status e = FMX_OK;
  PwTable pw = pw_table((int)A, &e);
  if (e) return e;
  if (A > 4096 && getenv("FMX_GROUP_SORTED") == nullptr) {
    // long rows: per-group compaction (moments) / per-group sort (rank) in one LDS buffer
    FMX_ARG(A <= 16384, "group ops hold one row in registers: A <= 16384");
    // rank: (key, asset) pairs of the largest group, sorted in LDS (<= 8192 members)
    int P = 2;
    while (P < A) P <<= 1;
    int Pmax = op == FMX_GROUP_RANK ? std::min(P, 8192) : (int)A;
    const size_t lds = op == FMX_GROUP_RANK ? (size_t)Pmax * 10 + 64 : (size_t)A * 8 + 64;
    const int E = (int)ceil_div(A, GL_NT);
#define FMX_GL(O) (E <= 5 ? (const void*)k_group_long<O, 5> : E <= 8 ? (const void*)k_group_long<O, 8> \
                           : E <= 12 ? (const void*)k_group_long<O, 12> : (const void*)k_group_long<O, 16>)
    const void* kl = op == FMX_GROUP_MEAN ? FMX_GL(0) : op == FMX_GROUP_NEUTRALIZE ? FMX_GL(1)
                   : op == FMX_GROUP_NORMALIZE ? FMX_GL(2) : FMX_GL(3);
#undef FMX_GL
    if ((e = set_lds(kl, lds))) return e;
    int ng = ngroups, m = method;
    void* args[] = {(void*)&X, (void*)&G, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&ng, (void*)&m,
                    (void*)&present, (void*)&pw, (void*)&Pmax};
    FMX_HIP(hipLaunchKernel(kl, dim3((unsigned)D, (unsigned)F), dim3(GL_NT), args, lds, as_stream(stream)));
    return FMX_OK;
  }
  int P = next_pow2((int)A);
  if (P < 2) P = 2;
  size_t lds = (size_t)P * 12 + 16 + (size_t)P * 8 + (2 * (P / 64) + 8) * 8 + 16 * 4 + (ngroups + 1) * 4 + 64;
  const void* k = op == FMX_GROUP_MEAN ? (const void*)k_group<0>
                : op == FMX_GROUP_NEUTRALIZE ? (const void*)k_group<1>
                : op == FMX_GROUP_NORMALIZE ? (const void*)k_group<2>
                                            : (const void*)k_group<3>;
  if ((e = set_lds(k, lds))) return e;
  int ng = ngroups, m = method;
  void* args[] = {(void*)&X, (void*)&G, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&P, (void*)&ng,
                  (void*)&m, (void*)&present, (void*)&pw};
  FMX_HIP(hipLaunchKernel(k, dim3((unsigned)D, (unsigned)F), dim3(CS_NT), args, lds, as_stream(stream)));
  return FMX_OK;
}

extern "C" fmx_status fmx_cs_regression(const double* Yv, const double* Xv, double* Out, int64_t D, int64_t A,
                                        int64_t ld, int32_t rettype, const uint8_t* present, void* stream) {
  FMX_ARG(Yv && Xv && Out, "null panel");
  FMX_ARG(D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  FMX_ARG(rettype >= 0 && rettype <= 4, "rettype");
  if (D == 0 || A == 0) return FMX_OK;
  fmx_status e = FMX_OK;
  PwTable pw = pw_table((int)A, &e);
  if (e) return e;
  size_t lds = (size_t)A * 16 + ((A * 2 + 15) & ~15) + (2 * (A / 64) + 8) * 8 + 16 * 4 + 64;
  if ((e = set_lds((const void*)k_cs_regression, lds))) return e;
  int rt = rettype;
  void* args[] = {(void*)&Yv, (void*)&Xv, (void*)&Out, (void*)&D, (void*)&A, (void*)&ld, (void*)&rt,
                  (void*)&present, (void*)&pw};
  FMX_HIP(hipLaunchKernel((const void*)k_cs_regression, dim3((unsigned)D), dim3(CS_NT), args, lds,
                          as_stream(stream)));
  return FMX_OK;
}

extern "C" fmx_status fmx_elementwise(int32_t op, const double* X, double* Y, int64_t n, double a, double b,
                                      void* stream) {
  FMX_ARG(X && Y && n >= 0, "bad args");
  FMX_ARG(op >= FMX_EW_SIGN && op <= FMX_EW_WHERE, "unknown elementwise op");
  if (n == 0) return FMX_OK;
  int grid = (int)std::min<int64_t>(ceil_div(n, 256), 8192);
  k_elementwise<<<grid, 256, 0, as_stream(stream)>>>(X, Y, n, op, a, b);
  FMX_LAUNCH_CHECK("k_elementwise");
  return FMX_OK;
}

extern "C" fmx_status fmx_bucket(const double* X, int32_t* codes, int64_t n, const double* edges,
                                 int32_t n_edges, void* stream) {
  FMX_ARG(X && codes && edges && n >= 0 && n_edges >= 2, "bad args");
  if (n == 0) return FMX_OK;
  int grid = (int)std::min<int64_t>(ceil_div(n, 256), 8192);
  k_bucket<<<grid, 256, 0, as_stream(stream)>>>(X, codes, n, edges, n_edges);
  FMX_LAUNCH_CHECK("k_bucket");
  return FMX_OK;
}
