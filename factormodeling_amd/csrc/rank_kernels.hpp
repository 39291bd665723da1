// Bucket-rank kernel templates (bucketrank.hpp): cs_rank (average/min/max/propagate), cs_winsor /
// cs_filter_center quantiles, and the fused two-lag daily IC.
//
// Reference: operations.py:54-75 (cs_rank, cs_winsor, cs_filter_center) and
// factor_selector.py:36-48 (per-date pearsonr, pearsonr(rankdata), beta).
//
// One 512-thread workgroup per row; every element stays in the registers of the thread
// that loaded it (key + one packed int of bucket/slot/mask), so outputs are written
// coalesced by their owner and no per-element index array lives in LDS.
#pragma once
#include "bucketrank.hpp"

namespace fmx {

// Development-only phase timer (make prof): thread 0 of every workgroup adds the wall
// time (100 MHz ticks) of each kernel phase to br_phase_acc[phase].
#ifdef FMX_PHASE_PROF
static __device__ unsigned long long br_phase_acc[32];
#define BR_PH_INIT uint64_t br_ph_t = wall_clock64(); int br_ph_i = 0
#define BR_PH()                                                                        \
  do {                                                                                 \
    if (threadIdx.x == 0) {                                                            \
      const uint64_t n_ = wall_clock64();                                              \
      atomicAdd(&br_phase_acc[br_ph_i & 31], (unsigned long long)(n_ - br_ph_t));      \
      br_ph_t = n_;                                                                    \
    }                                                                                  \
    ++br_ph_i;                                                                         \
  } while (0)
#define BR_PH_ROW() br_ph_i = 0
#define BR_PH_PARAMS , uint64_t &br_ph_t, int &br_ph_i     // phase state into a device helper
#define BR_PH_ARGS , br_ph_t, br_ph_i
#define BR_PHASE_EXPORT(NAME)                                                          \
  extern "C" int NAME(unsigned long long* out) {                                       \
    unsigned long long z[32] = {};                                                     \
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(fmx::br_phase_acc), sizeof(z)) != hipSuccess) return 1; \
    return hipMemcpyToSymbol(HIP_SYMBOL(fmx::br_phase_acc), z, sizeof(z)) != hipSuccess;     \
  }
#else
#define BR_PH_INIT (void)0
#define BR_PH() (void)0
#define BR_PH_ROW() (void)0
#define BR_PH_PARAMS
#define BR_PH_ARGS
#define BR_PHASE_EXPORT(NAME)
#endif

// packed per-element state: slot (14 bits) | bucket << 14 (12 bits) | mask << 26
constexpr int PK_SLOT = 0x3fff;
constexpr int PK_BSHIFT = 14;
constexpr int PK_BMASK = 0xfff;
constexpr int PK_MSHIFT = 26;

// In-bucket counts of keys < key and == key among the bucketed members [s0, s1).
__device__ __forceinline__ void br_count(const uint64_t* bkey, int s0, int s1, uint64_t key, int* lt, int* eq) {
  int l = 0, e = 0;
#pragma unroll 4
  for (int q = s0; q < s1; ++q) {
    const uint64_t y = bkey[q];
    l += y < key;
    e += y == key;
  }
  *lt = l;
  *eq = e;
}

// ------------------------------------------------------------------------------------
// cs_rank: y = (rank - 1) / (len(row) - 1), len counting NaN rows; 0.5 for single-row
// dates (operations.py:58-60).  Rows are (f, d) = blockIdx.x / D, % D.
template <int NT, int EMAX>
__global__ void __launch_bounds__(NT)
k_cs_rank_br(const double* __restrict__ X, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld, int method,
             const uint8_t* __restrict__ present) {
  constexpr int BR_NT = NT, BR_NS = BRG<NT>::NS, BR_NB = BRG<NT>::NB, BR_NW = BRG<NT>::NW;
  (void)BR_NS;
  __shared__ uint64_t spl[BR_NS];
  __shared__ int cnt[BR_NB + 1];
  __shared__ int iscr[2 * (BR_NW + 1)];
  extern __shared__ uint64_t bkey[];          // max(A, NT) keys
  const int t = threadIdx.x;
  BR_PH_INIT;
  const int64_t row = fmx_blk();              // grid dim3(D, F)
  const int64_t d = row % D;
  const double* x = X + row * ld;
  double* y = Y + row * ld;
  const uint8_t* prow = present ? present + d * ld : nullptr;
  uint64_t key[EMAX];
  int pk[EMAX];
  int nl = 0;                                 // present | valid << 16
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t i = t + (int64_t)k * BR_NT;
    key[k] = KEY_SENTINEL;
    if (i < A) {
      const bool p = prow ? prow[i] != 0 : true;
      const double v = x[i];
      nl += p;
      if (p && v == v) { key[k] = okey(v); nl += 1 << 16; }
    }
  }
  for (int b = t; b <= BR_NB; b += BR_NT) cnt[b] = 0;
  br_sum<NT, 1, int>(&nl, iscr);
  BR_PH();
  const int nrow = nl & 0xffff, nv = nl >> 16;
  if (method == FMX_RANK_AVERAGE_PROPAGATE && nv < nrow) {
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const int64_t i = t + (int64_t)k * BR_NT;
      if (i < A) y[i] = qnan();
    }
    return;
  }
  const bool half = (method != FMX_RANK_AVERAGE_PROPAGATE) && nrow == 1;
  if (half || nv == 0) {
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const int64_t i = t + (int64_t)k * BR_NT;
      if (i < A) {
        const bool p = prow ? prow[i] != 0 : true;
        y[i] = (p && half) ? 0.5 : qnan();
      }
    }
    return;
  }
  br_splitters<NT>(spl, bkey, br_sample<NT>(x, prow, A));
  BR_PH();
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    if (key[k] != KEY_SENTINEL) {
      const int b = br_bucket<NT>(spl, key[k]);
      pk[k] = atomicAdd(&cnt[b], 1) | (b << PK_BSHIFT);
    }
  }
  __syncthreads();
  br_scan<NT, 1>(cnt, 0, iscr);
  BR_PH();
#pragma unroll
  for (int k = 0; k < EMAX; ++k)
    if (key[k] != KEY_SENTINEL) bkey[cnt[pk[k] >> PK_BSHIFT] + (pk[k] & PK_SLOT)] = key[k];
  __syncthreads();
  BR_PH();
  const double den = (double)(nrow - 1);
  // in-bucket counts of all EMAX elements in one interleaved loop (independent LDS
  // reads per iteration): le[k] = #less | #equal << 16 among the bucket's members
  int s0[EMAX], len[EMAX], le[EMAX];
  int maxlen = 0;
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    s0[k] = 0; len[k] = 0; le[k] = 0;
    if (key[k] == KEY_SENTINEL) continue;
    const int b = pk[k] >> PK_BSHIFT;
    s0[k] = cnt[b];
    const int n = cnt[b + 1] - s0[k];
    if (b & 1) le[k] = n << 16; else len[k] = n;
    maxlen = max(maxlen, len[k]);
  }
  for (int j = 0; j < maxlen; ++j) {
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (j < len[k]) {
        const uint64_t w = bkey[s0[k] + j];
        le[k] += (w < key[k]) + ((w == key[k]) << 16);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t i = t + (int64_t)k * BR_NT;
    if (i >= A) continue;
    if (key[k] == KEY_SENTINEL) { y[i] = qnan(); continue; }
    const int lt = le[k] & 0xffff, eq = le[k] >> 16;
    const int less = s0[k] + lt;
    double r;
    if (method == FMX_RANK_MIN) r = (double)(less + 1);
    else if (method == FMX_RANK_MAX) r = (double)(less + eq);
    else r = (double)less + (double)(eq + 1) / 2.0;
    y[i] = (r - 1.0) / den;
  }
  BR_PH();
}

// ------------------------------------------------------------------------------------
// OP 0 = cs_winsor (clip to the quantiles when >= 5 non-NaN), 1 = cs_filter_center.
// Quantiles are numpy 'linear' percentiles from order statistics; the order statistic k
// lies in the bucket b with start[b] <= k < start[b+1]: a splitter value when b is an
// equal-bucket, otherwise the (k - start[b])-th smallest of that bucket's few members,
// which are gathered into a short LDS list (or, if a bucket is pathologically large,
// found by bisection of the key space with block counts).
constexpr int QCAP = 512;

template <int OP, int NT, int EMAX>
__global__ void __launch_bounds__(NT)
k_cs_quantile_br(const double* __restrict__ X, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld,
                 double qlo, double qhi, const uint8_t* __restrict__ present) {
  constexpr int BR_NT = NT, BR_NS = BRG<NT>::NS, BR_NB = BRG<NT>::NB, BR_NW = BRG<NT>::NW;
  (void)BR_NS;
  __shared__ uint64_t spl[BR_NS];
  __shared__ int cnt[BR_NB + 1];
  __shared__ int iscr[2 * (BR_NW + 1)];
  __shared__ int tfill[4];
  __shared__ uint64_t tval[4];
  extern __shared__ uint64_t lists[];         // 4 * QCAP keys (also splitter scratch)
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  BR_PH_INIT;
  const int64_t row = fmx_blk();              // grid dim3(D, F)
  const int64_t d = row % D;
  const double* x = X + row * ld;
  double* y = Y + row * ld;
  const uint8_t* prow = present ? present + d * ld : nullptr;
  uint64_t key[EMAX];
  int bk[EMAX];
  int nv = 0;
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t i = t + (int64_t)k * BR_NT;
    key[k] = KEY_SENTINEL;
    if (i < A && (prow ? prow[i] != 0 : true)) {
      const double v = x[i];
      if (v == v) { key[k] = okey(v); nv += 1; }
    }
  }
  for (int b = t; b <= BR_NB; b += BR_NT) cnt[b] = 0;
  if (t < 4) tfill[t] = 0;
  br_sum<NT, 1, int>(&nv, iscr);
  double lo = qnan(), hi = qnan();
  if (nv > 0 && (OP == 1 || nv >= 5)) {
    br_splitters<NT>(spl, lists, br_sample<NT>(x, prow, A));
    BR_PH();
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      bk[k] = -1;
      if (key[k] != KEY_SENTINEL) {
        bk[k] = br_bucket<NT>(spl, key[k]);
        atomicAdd(&cnt[bk[k]], 1);
      }
    }
    __syncthreads();
    br_scan<NT, 1>(cnt, 0, iscr);
    BR_PH();
    // order statistics: (p, p+1) per quantile (numpy linear), identical when vi >= n-1
    const double qs[2] = {qlo, qhi};
    double gq[2];
    int kk[4];
    bool top[2];
#pragma unroll
    for (int z = 0; z < 2; ++z) {
      const double vi = (double)(nv - 1) * qs[z];
      top[z] = vi >= (double)(nv - 1);
      if (top[z]) {
        kk[2 * z] = kk[2 * z + 1] = nv - 1;
        gq[z] = vi + 1.0;
      } else {
        const double pf = floor(vi);
        kk[2 * z] = (int)pf;
        kk[2 * z + 1] = (int)pf + 1;
        gq[z] = vi - pf;
      }
    }
    int tb[4];
    bool slow = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int l = 0, h = BR_NB + 1;                // last b with cnt[b] <= k
      while (l < h) { const int m = (l + h) >> 1; if (cnt[m] <= kk[j]) l = m + 1; else h = m; }
      tb[j] = l - 1;
      slow |= !(tb[j] & 1) && (cnt[tb[j] + 1] - cnt[tb[j]]) > QCAP;
    }
    BR_PH();
    if (!slow) {
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
        if (bk[k] < 0 || (bk[k] & 1)) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (bk[k] == tb[j]) lists[j * QCAP + atomicAdd(&tfill[j], 1)] = key[k];
      }
      __syncthreads();
      if (wid < 4) {
        const int j = wid, b = tb[j];
        if (b & 1) {
          if (lane == 0) tval[j] = spl[b >> 1];
        } else {
          const uint64_t* L = lists + j * QCAP;
          const int n = cnt[b + 1] - cnt[b], r = kk[j] - cnt[b];
          for (int q = lane; q < n; q += 64) {
            int lt, eq;
            br_count(L, 0, n, L[q], &lt, &eq);
            if (lt <= r && r < lt + eq) tval[j] = L[q];   // all writers store the same key
          }
        }
      }
      __syncthreads();
    } else {
      // bisection: smallest key v with #{keys <= v} > k
      for (int j = 0; j < 4; ++j) {
        uint64_t l = 0, h = KEY_SENTINEL - 1;
        while (l < h) {
          const uint64_t m = l + ((h - l) >> 1);
          int c = 0;
#pragma unroll
          for (int k = 0; k < EMAX; ++k) c += key[k] <= m;   // sentinel > m always
          br_sum<NT, 1, int>(&c, iscr);
          if (c > kk[j]) h = m; else l = m + 1;
        }
        if (t == 0) tval[j] = l;
      }
      __syncthreads();
    }
    BR_PH();
    double qv[2];
#pragma unroll
    for (int z = 0; z < 2; ++z) {
      const double a = okey_inv(tval[2 * z]), b = okey_inv(tval[2 * z + 1]);
      const double g = gq[z];
      const double diff = b - a;
      qv[z] = (g >= 0.5) ? b - diff * (1.0 - g) : a + diff * g;
    }
    lo = qv[0];
    hi = qv[1];
  }
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t i = t + (int64_t)k * BR_NT;
    if (i >= A) continue;
    if (prow && !prow[i]) { y[i] = qnan(); continue; }
    const double v = key[k] == KEY_SENTINEL ? qnan() : okey_inv(key[k]);
    double o;
    if (OP == 0) {
      o = v;
      if (nv >= 5) o = (v < lo) ? lo : ((v > hi) ? hi : v);
    } else {
      o = (v < lo || v > hi) ? v : 0.0;
    }
    y[i] = o;
  }
}

// ------------------------------------------------------------------------------------
// Fused daily IC: workgroup (source row s, factor f) ranks X[f][s] once and produces the
// stats of the pairs (X[f][s], R[s + L_m]) for up to two lags.  Members of the bucketing
// are the exposures that are pair-valid for at least one lag; mask bit m marks lag m.
// Per-lag bucket counts are packed 16|16 in one int array and scanned together.
// Output: out[((m*4 + j) * F + f) * D + s + L_m], j = n, IC, rank IC, beta.
template <int NT, int EMAX>
__global__ void __launch_bounds__(NT, NT == 1024 ? 8 : 4)
k_ic_daily_br(const double* __restrict__ X, const double* __restrict__ Rt, int64_t F, int64_t D, int64_t A,
              int64_t ld, int L0, int L1, int NL, double* __restrict__ out) {
  constexpr int BR_NT = NT, BR_NS = BRG<NT>::NS, BR_NB = BRG<NT>::NB, BR_NW = BRG<NT>::NW;
  (void)BR_NS;
  __shared__ uint64_t spl[BR_NS];
  __shared__ int cnt[2][BR_NB + 1];
  __shared__ int iscr[2 * (BR_NW + 1)];
  __shared__ double dscr[(BR_NW + 1) * 14];
  extern __shared__ uint64_t bkey[];          // max(A, NT) keys, then A mask bytes
  const int64_t kcap = A > BR_NT ? A : BR_NT;
  uint8_t* bmask = (uint8_t*)(bkey + kcap);
  const int t = threadIdx.x;
  BR_PH_INIT;
  const int64_t s = fmx_blk() / F, f = fmx_blk() % F;   // grid dim3(F, D)
  const double* xf = X + (f * D + s) * ld;
  const int lagv[2] = {L0, L1};
  const double* rr[2];
  bool act[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    act[m] = m < NL && s + lagv[m] < D;
    rr[m] = act[m] ? Rt + (s + lagv[m]) * ld : nullptr;
  }
  if (!act[0] && !act[1]) return;
  uint64_t key[EMAX];
  int pk[EMAX];
  // v1: n per lag, sum f per lag, sum r per lag;  mx: -min f, max f, -min r, max r per lag
  double v1[6] = {0, 0, 0, 0, 0, 0};
  double mx[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) mx[q] = -INFINITY;
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t i = t + (int64_t)k * BR_NT;
    key[k] = KEY_SENTINEL;
    pk[k] = 0;
    if (i < A) {
      const double v = xf[i];
      if (v == v) {
        int mm = 0;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          if (!act[m]) continue;
          const double r = rr[m][i];
          if (r != r) continue;
          mm |= 1 << m;
          v1[m] += 1.0;
          v1[2 + 2 * m] += v;
          v1[3 + 2 * m] += r;
          mx[4 * m + 0] = fmax(mx[4 * m + 0], -v);
          mx[4 * m + 1] = fmax(mx[4 * m + 1], v);
          mx[4 * m + 2] = fmax(mx[4 * m + 2], -r);
          mx[4 * m + 3] = fmax(mx[4 * m + 3], r);
        }
        if (mm) { key[k] = okey(v); pk[k] = mm << PK_MSHIFT; }
      }
    }
  }
  for (int b = t; b <= BR_NB; b += BR_NT) { cnt[0][b] = 0; cnt[1][b] = 0; }
  br_part<6, false>(v1, dscr, 14, 0);
  br_part<8, true>(mx, dscr, 14, 6);
  br_fin<NT>(dscr, 14, 6);
  const double* tot1 = dscr + BR_NW * 14;      // sums [0,6), -min/max [6,14)
#pragma unroll
  for (int q = 0; q < 6; ++q) v1[q] = tot1[q];
  BR_PH();
  __shared__ double cst[8];                   // only thread 0 reads them back
  if (t == 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) cst[q] = tot1[6 + q];
  }
  const int n[2] = {(int)v1[0], (int)v1[1]};
  const bool need = (act[0] && n[0] >= 3) || (act[1] && n[1] >= 3);
  __shared__ double fin[14];                  // per-lag moment totals (thread 0)
  if (need) {
    br_splitters<NT>(spl, bkey, br_sample<NT>(xf, nullptr, A));
    BR_PH();
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (key[k] != KEY_SENTINEL) {
        const int b = br_bucket<NT>(spl, key[k]);
        const int mm = pk[k] >> PK_MSHIFT;
        pk[k] |= atomicAdd(&cnt[0][b], 1) | (b << PK_BSHIFT);
        atomicAdd(&cnt[1][b], (mm & 1) | ((mm >> 1) << 16));
      }
    }
    __syncthreads();
    br_scan<NT, 2>(&cnt[0][0], BR_NB + 1, iscr);
    BR_PH();
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (key[k] == KEY_SENTINEL) continue;
      const int q = cnt[0][(pk[k] >> PK_BSHIFT) & PK_BMASK] + (pk[k] & PK_SLOT);
      bkey[q] = key[k];
      bmask[q] = (uint8_t)(pk[k] >> PK_MSHIFT);
    }
    __syncthreads();
    BR_PH();
    // ranks: pk[k] <- 2*rank(lag 0) | 2*rank(lag 1) << 16 (half-integer ranks, exact);
    // the mask moves to bit 31/30 of a separate int
    int msk[EMAX];
    // in-bucket counts per lag in one interleaved loop over the EMAX elements:
    // a0[k] = lt | eq << 16 among the bucket's lag-0 members, a1[k] the same for lag 1
    int s0[EMAX], len[EMAX], a0[EMAX], a1[EMAX];
    int maxlen = 0;
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      msk[k] = 0; s0[k] = 0; len[k] = 0; a0[k] = 0; a1[k] = 0;
      if (key[k] == KEY_SENTINEL) continue;
      const int b = (pk[k] >> PK_BSHIFT) & PK_BMASK;
      msk[k] = pk[k] >> PK_MSHIFT;
      s0[k] = cnt[0][b];
      if (b & 1) {
        const int c0 = cnt[1][b], c1 = cnt[1][b + 1];
        a0[k] = ((c1 & 0xffff) - (c0 & 0xffff)) << 16;
        a1[k] = ((c1 >> 16) - (c0 >> 16)) << 16;
      } else {
        len[k] = cnt[0][b + 1] - s0[k];
      }
      maxlen = max(maxlen, len[k]);
    }
    for (int j = 0; j < maxlen; ++j) {
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
        if (j < len[k]) {
          const uint64_t w = bkey[s0[k] + j];
          const int wm = bmask[s0[k] + j];
          const int inc = (w < key[k]) + ((w == key[k]) << 16);
          a0[k] += (wm & 1) ? inc : 0;
          a1[k] += (wm & 2) ? inc : 0;
        }
      }
    }
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (key[k] == KEY_SENTINEL) continue;
      const int c0 = cnt[1][(pk[k] >> PK_BSHIFT) & PK_BMASK];
      // 2*rank = 2*(base + lt) + eq + 1
      pk[k] = (2 * ((c0 & 0xffff) + (a0[k] & 0xffff)) + (a0[k] >> 16) + 1) |
              ((2 * ((c0 >> 16) + (a1[k] & 0xffff)) + (a1[k] >> 16) + 1) << 16);
    }
    double fm[2], rm[2], km[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const double dn = (double)n[m];
      fm[m] = v1[2 + 2 * m] / dn;
      rm[m] = v1[3 + 2 * m] / dn;
      km[m] = (dn + 1.0) / 2.0;
    }
    BR_PH();
    // one lag at a time keeps 7 accumulators live; thread 0 parks the totals in LDS
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      double w[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
        if (!((msk[k] >> m) & 1)) continue;
        const int64_t i = t + (int64_t)k * BR_NT;
        const double fv = okey_inv(key[k]);
        const int r2 = m == 0 ? (pk[k] & 0xffff) : (int)((unsigned)pk[k] >> 16);
        const double rk = (double)r2 / 2.0;
        const double r = rr[m][i];
        const double dx = fv - fm[m], dy = r - rm[m], dk = rk - km[m];
        w[0] += dx * dy; w[1] += dx * dx; w[2] += dy * dy;
        w[3] += dk * dy; w[4] += dk * dk;
        w[5] += fv * fv; w[6] += fv * r;
      }
      br_part<7, false>(w, dscr, 14, 7 * m);
    }
    br_fin<NT>(dscr, 14, 14);
    if (t < 14) fin[t] = dscr[BR_NW * 14 + t];
    __syncthreads();
  }
  if (t == 0) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      if (!act[m]) continue;
      const int64_t td = s + lagv[m];
      double* o = out + ((int64_t)(m * 4) * F + f) * D + td;
      const int64_t st = F * D;
      const int nn = n[m];
      double ic = qnan(), ric = qnan(), beta = qnan();
      if (nn >= 3) {
        const double* w = fin + 7 * m;
        const bool fconst = (-cst[4 * m + 0]) == cst[4 * m + 1];
        const bool rconst = (-cst[4 * m + 2]) == cst[4 * m + 3];
        if (!fconst && !rconst) {
          ic = fmin(1.0, fmax(-1.0, w[0] / sqrt(w[1] * w[2])));
          ric = fmin(1.0, fmax(-1.0, w[3] / sqrt(w[4] * w[2])));
        }
        beta = w[5] > 0 ? w[6] / w[5] : qnan();
      }
      o[0] = (double)nn;
      o[st] = ic;
      o[2 * st] = ric;
      o[3 * st] = beta;
    }
  }
  BR_PH();
}

}  // namespace fmx
