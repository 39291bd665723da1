// Fine-bucket rank kernels (finerank.hpp): cs_rank and the fused two-lag daily IC.
//
// Reference: operations.py:54-62 (cs_rank: pandas Series.rank) and
// factor_selector.py:36-48 (per-date pearsonr, pearsonr(rankdata), beta).
//
// One workgroup of NT threads per row; thread t owns row positions t + k*NT (k < EMAX)
// in registers, so loads and stores are coalesced by their owner.  Per row: one global
// read, one block reduction (counts, min, max), a 64-key wave sort, one LDS atomic per
// element into ~65*(K+1) bucket counters, a block scan of the counters, and an in-bucket
// scan only for elements that share a fine bucket.
#pragma once
#include "finerank.hpp"
#include "rank_kernels.hpp"

namespace fmx {

constexpr int FR_K_CS = 127;   // fine buckets per interval (cs_rank: 33 KB of int counters)
constexpr int FR_K_IC = 62;    // (IC: 64-bit packed counters, 32 KB: two rows fit a CU)

// ------------------------------------------------------------------------------------
// cs_rank: y = (rank - 1) / (len(row) - 1), len counting NaN rows; 0.5 for single-row
// dates (operations.py:58-60).  Rows are (f, d) = blockIdx.x / D, % D.
template <int NT, int EMAX>
__global__ void __launch_bounds__(NT)
k_cs_rank_fr(const double* __restrict__ X, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld, int method,
             const uint8_t* __restrict__ present) {
  constexpr int K = FR_K_CS, NB = FRG<K>::NB, NW = NT / 64;
  __shared__ FrTab tab;
  __shared__ int cnt[NB + 1];
  __shared__ double dscr[(NW + 1) * 4];
  __shared__ int iscr[NW];
  extern __shared__ uint64_t bkey[];          // A keys
  const int t = threadIdx.x, wid = t >> 6;
  BR_PH_INIT;
  const int64_t row = blockIdx.x;
  const int64_t d = row % D;
  const double* x = X + row * ld;
  double* y = Y + row * ld;
  const uint8_t* prow = present ? present + d * ld : nullptr;
  uint64_t key[EMAX];
  double st[4] = {0.0, 0.0, -INFINITY, -INFINITY};   // nrow, nvalid, -min, max
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t i = t + (int64_t)k * NT;
    key[k] = KEY_SENTINEL;
    if (i < A) {
      const bool p = prow ? prow[i] != 0 : true;
      const double v = x[i];
      st[0] += p;
      if (p && v == v) {
        key[k] = okey(v);
        st[1] += 1.0;
        st[2] = fmax(st[2], -v);
        st[3] = fmax(st[3], v);
      }
    }
  }
  const uint64_t smp = wid == 0 ? fr_sample(x, prow, A) : KEY_SENTINEL;
  for (int b = t; b <= NB; b += NT) cnt[b] = 0;
  br_part<2, false>(st, dscr, 4, 0);
  br_part<2, true>(st + 2, dscr, 4, 2);
  br_fin<NT>(dscr, 4, 2);
  const int nrow = (int)dscr[NW * 4 + 0], nv = (int)dscr[NW * 4 + 1];
  const double vmin = -dscr[NW * 4 + 2], vmax = dscr[NW * 4 + 3];
  BR_PH();
  if (method == FMX_RANK_AVERAGE_PROPAGATE && nv < nrow) {
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const int64_t i = t + (int64_t)k * NT;
      if (i < A) y[i] = qnan();
    }
    return;
  }
  const bool half = (method != FMX_RANK_AVERAGE_PROPAGATE) && nrow == 1;
  if (half || nv == 0) {
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const int64_t i = t + (int64_t)k * NT;
      if (i < A) {
        const bool p = prow ? prow[i] != 0 : true;
        y[i] = (p && half) ? 0.5 : qnan();
      }
    }
    return;
  }
  if (wid == 0) fr_build_w0<K>(tab, smp, vmin, vmax);
  __syncthreads();
  BR_PH();
  int pk[EMAX];                               // slot | bucket << PK_BSHIFT
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    if (key[k] != KEY_SENTINEL) {
      const int b = fr_bucket<K>(tab, key[k], okey_inv(key[k]));
      pk[k] = atomicAdd(&cnt[b], 1) | (b << PK_BSHIFT);
    }
  }
  __syncthreads();
  fr_scan<NT, int>(cnt, NB, iscr);
  BR_PH();
  // le[k] = #less | #equal << 16 inside the bucket; only shared fine buckets need the scan
  int s0[EMAX], len[EMAX], le[EMAX];
  int maxlen = 0;
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    s0[k] = 0; len[k] = 0; le[k] = 0;
    if (key[k] == KEY_SENTINEL) continue;
    const int b = pk[k] >> PK_BSHIFT;
    s0[k] = cnt[b];
    const int n = cnt[b + 1] - s0[k];
    if ((b % (K + 1)) == K) le[k] = n << 16;           // equal-to-sample bucket
    else if (n == 1) le[k] = 1 << 16;
    else {
      len[k] = n;
      bkey[s0[k] + (pk[k] & PK_SLOT)] = key[k];
    }
    maxlen = max(maxlen, len[k]);
  }
  __syncthreads();
  BR_PH();
  for (int j = 0; j < maxlen; ++j) {
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (j < len[k]) {
        const uint64_t w = bkey[s0[k] + j];
        le[k] += (w < key[k]) + ((w == key[k]) << 16);
      }
    }
  }
  const double den = (double)(nrow - 1);
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t i = t + (int64_t)k * NT;
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
// Fused daily IC: workgroup (source row s, factor f) ranks X[f][s] once and produces the
// stats of the pairs (X[f][s], R[s + L_m]) for up to two lags.  Bucket members are the
// exposures pair-valid for at least one lag; one 64-bit counter per bucket packs
// (#members | #lag-0 members << 16 | #lag-1 members << 32), so a single atomic gives the
// scatter slot and a single scan gives both lags' rank bases.
// Output: out[((m*4 + j) * F + f) * D + s + L_m], j = n, IC, rank IC, beta.
template <int NT, int EMAX>
__global__ void __launch_bounds__(NT, NT == 1024 ? 8 : 4)
k_ic_daily_fr(const double* __restrict__ X, const double* __restrict__ Rt, int64_t F, int64_t D, int64_t A,
              int64_t ld, int L0, int L1, int NL, double* __restrict__ out) {
  constexpr int K = FR_K_IC, NB = FRG<K>::NB, NW = NT / 64;
  // packed per-element state: slot (14 bits) | bucket << 14 (13 bits) | lag mask << 27
  constexpr int FR_MSH = 27, FR_BMASK = 0x1fff;
  static_assert(NB <= FR_BMASK, "bucket id field");
  using u64 = unsigned long long;
  __shared__ FrTab tab;
  __shared__ u64 cnt[NB + 1];
  __shared__ u64 uscr[NW];
  __shared__ double dscr[(NW + 1) * 14];
  extern __shared__ uint64_t bkey[];          // A keys, then A mask bytes
  uint8_t* bmask = (uint8_t*)(bkey + A);
  const int t = threadIdx.x, wid = t >> 6;
  BR_PH_INIT;
  const int64_t s = blockIdx.x / F, f = blockIdx.x % F;
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
  int pk[EMAX];                               // mask << FR_MSH, later slot | bucket
  // v1: n per lag, sum f per lag, sum r per lag;  mx: -min f, max f, -min r, max r per lag
  double v1[6] = {0, 0, 0, 0, 0, 0};
  double mx[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) mx[q] = -INFINITY;
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t i = t + (int64_t)k * NT;
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
        if (mm) { key[k] = okey(v); pk[k] = mm << FR_MSH; }
      }
    }
  }
  const uint64_t smp = wid == 0 ? fr_sample(xf, nullptr, A) : KEY_SENTINEL;
  for (int b = t; b <= NB; b += NT) cnt[b] = 0;
  br_part<6, false>(v1, dscr, 14, 0);
  br_part<8, true>(mx, dscr, 14, 6);
  br_fin<NT>(dscr, 14, 6);
  const double* tot1 = dscr + NW * 14;        // sums [0,6), -min/max [6,14)
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
    if (wid == 0) {
      // bounds of the union of both lags' members (empty lag: -min = max = -inf)
      const double vmin = -fmax(tot1[6], tot1[10]), vmax = fmax(tot1[7], tot1[11]);
      fr_build_w0<K>(tab, smp, vmin, vmax);
    }
    __syncthreads();
    BR_PH();
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (key[k] != KEY_SENTINEL) {
        const int b = fr_bucket<K>(tab, key[k], okey_inv(key[k]));
        const int mm = pk[k] >> FR_MSH;
        const u64 inc = 1ull | ((u64)(mm & 1) << 16) | ((u64)(mm >> 1) << 32);
        const u64 old = atomicAdd(&cnt[b], inc);
        pk[k] |= (int)(old & 0xffff) | (b << PK_BSHIFT);
      }
    }
    __syncthreads();
    fr_scan<NT, u64>(cnt, NB, uscr);
    BR_PH();
    // a0[k] / a1[k] = #less | #equal << 16 among the bucket's lag-0 / lag-1 members
    int msk[EMAX], s0[EMAX], len[EMAX], a0[EMAX], a1[EMAX];
    int maxlen = 0;
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      msk[k] = 0; s0[k] = 0; len[k] = 0; a0[k] = 0; a1[k] = 0;
      if (key[k] == KEY_SENTINEL) continue;
      const int b = (pk[k] >> PK_BSHIFT) & FR_BMASK;
      msk[k] = pk[k] >> FR_MSH;
      const u64 c0 = cnt[b], dc = cnt[b + 1] - c0;
      const int nall = (int)(dc & 0xffff);
      s0[k] = (int)(c0 & 0xffff);
      if ((b % (K + 1)) == K) {
        a0[k] = (int)((dc >> 16) & 0xffff) << 16;
        a1[k] = (int)((dc >> 32) & 0xffff) << 16;
      } else if (nall == 1) {
        a0[k] = (msk[k] & 1) << 16;
        a1[k] = (msk[k] >> 1) << 16;
      } else {
        len[k] = nall;
        const int q = s0[k] + (pk[k] & PK_SLOT);
        bkey[q] = key[k];
        bmask[q] = (uint8_t)msk[k];
      }
      maxlen = max(maxlen, len[k]);
    }
    __syncthreads();
    BR_PH();
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
    // pk[k] <- 2*rank(lag 0) | 2*rank(lag 1) << 16 (half-integer ranks, exact)
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (key[k] == KEY_SENTINEL) continue;
      const u64 c0 = cnt[(pk[k] >> PK_BSHIFT) & FR_BMASK];
      const int b0 = (int)((c0 >> 16) & 0xffff), b1 = (int)((c0 >> 32) & 0xffff);
      pk[k] = (2 * (b0 + (a0[k] & 0xffff)) + (a0[k] >> 16) + 1) |
              ((2 * (b1 + (a1[k] & 0xffff)) + (a1[k] >> 16) + 1) << 16);
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
    // one lag at a time keeps 7 accumulators live
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      double w[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
        if (!((msk[k] >> m) & 1)) continue;
        const int64_t i = t + (int64_t)k * NT;
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
    if (t < 14) fin[t] = dscr[NW * 14 + t];
    __syncthreads();
  }
  if (t == 0) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      if (!act[m]) continue;
      const int64_t td = s + lagv[m];
      double* o = out + ((int64_t)(m * 4) * F + f) * D + td;
      const int64_t stp = F * D;
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
      o[stp] = ic;
      o[2 * stp] = ric;
      o[3 * stp] = beta;
    }
  }
  BR_PH();
}

}  // namespace fmx
