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

// min waves per SIMD of the aliased-LDS cs_rank kernel: three rows per CU
#ifndef FR_FA_WAVES1024
#define FR_FA_WAVES1024 8
#endif
#ifndef FR_FA_WAVES
#define FR_FA_WAVES(NT) ((NT) == 1024 ? FR_FA_WAVES1024 : ((NT) == 640 ? 8 : 6))
#endif
// ... but no more than the LDS lets in: a row stages up to EMAX*NT 8-byte keys (at least
// the 32 KB counter array), so long rows (EMAX*NT > 6144) hold one or two rows per CU
// (two up to ~15/16 of EMAX*NT: C5's 10,000 assets in <1024,10>).  Asking for more waves
// than can be resident only caps the VGPRs and spills the key registers
// (k_cs_rank_fa<512,20>: 340 B/lane of scratch at a fixed 6-wave bound).
constexpr int fr_fa_min_waves(int nt, int emax) {
  const int dyn = emax * nt * 8 > 32768 ? emax * nt * 8 : 32768;
  const int rows = (160 * 1024) / (dyn / 16 * 15 + 2048);
  const int w = rows * nt / 256;
  return w < 1 ? 1 : (w > FR_FA_WAVES(nt) ? FR_FA_WAVES(nt) : w);
}
// Row slot k of thread t holds position t + k*NT.  br_emax rounds ceil(A / NT) up to the
// next instantiated EMAX (7 -> 8, 9 -> 10, 11 -> 12, 13..15 -> 16, ...), so any slot, not
// just the last, may lie past the row's end: every slot is tested, and the unconditional
// loads are clamped into the row.
template <int NT>
__device__ __forceinline__ bool fr_in(int t, int k, int A) { return t + k * NT < A; }
template <int NT>
__device__ __forceinline__ int fr_ix(int t, int k, int A) {
  const int i = t + k * NT;
  return i < A ? i : (A > 0 ? A - 1 : 0);
}
// Scheduling fence between unrolled per-element steps: bounds how many elements' live
// ranges overlap (register pressure at 8 waves/SIMD) -- other waves hide the latency.
#ifndef FR_NO_SCHED_FENCE
#define FR_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define FR_SCHED_FENCE() (void)0
#endif
// in-bucket scan of k_cs_rank_fa: one loop per element slot (1) or one loop over all (0)
#ifndef FR_SCAN_PERK
#define FR_SCAN_PERK 1
#endif
constexpr int FR_K_CS = 247;   // fine buckets per interval (cs_rank: 16-bit counters, 32 KB)
constexpr int FR_CS_WORDS = 8192;
constexpr int FR_K_IC = 62;    // (IC: 64-bit packed counters, 32 KB: two rows fit a CU)

// Daily IC fused into the rank pass (k_cs_rank_fa<..., IC = true>): the workgroup that
// ranks row (f, s) also reduces the pairs (X[f][s], R[s + L_m]) of up to two lags, so the
// ranks never leave the CU (factor_selector.py:36-48).  Rows run date-major (workgroup b
// -> s = b / F, f = b % F): the F rows of a date share its return rows in L2.
struct FrIc {
  const double* Rt;          // returns [D][ld]
  const uint32_t* nanb;      // NaN-return bits [D][nw] (k_ret_rows)
  const double* rsh;         // [D] first non-NaN return of each date (0 if none): moment anchor
  int64_t F, nw;
  int L0, L1, NL;
  double* out;               // [NL][4][F][D] = (n, IC, rank IC, beta) at target date s + L
  int32_t* ovf;              // [1 + F*D]: rows whose NaN-return list exceeds FR_IC_EC
  fmx_rank2_t* RK;           // the doubled ranks of those rows (k_ic_ranked_list input)
};
// cs_zscore + market_neutralize fused into the rank + winsor pass (k_cs_rank_fa<..., ZN>):
// the row's numpy moments from the same load (operations.py:77-78, :171-182).
struct FrZn {
  double* Yz;                // cs_zscore output
  double* Yn;                // market_neutralize output
  PwTable pw;                // numpy pairwise schedules (the row length's)
  int slen;                  // its length in int32 words
};
constexpr int FR_ZN_NODES = 2 * (16384 / 64) + 8;
// the moments' scratch (schedule + tree nodes) aliases the scan list: bytes it needs there
constexpr int FR_ZN_SCR_BYTES = PW_LDS_MAX * 4 + FR_ZN_NODES * 8;
constexpr int FR_IC_EC = 256;  // E entries per lag held in LDS; longer lists: ovf
#ifndef FR_IC_CH
#define FR_IC_CH 2             // return loads in flight per thread in the IC pass
#endif

struct FrIcRow {
  int64_t s, f;              // source date, factor
  int lag[2];
  bool act[2];               // lag m has a target date s + L_m < D
};

__device__ __forceinline__ FrIcRow fr_ic_row(const FrIc& ic, int64_t D) {
  FrIcRow r;
  r.s = fmx_blk() / ic.F;                     // grid dim3(F, D): date-major rows
  r.f = fmx_blk() % ic.F;
  r.lag[0] = ic.L0;
  r.lag[1] = ic.L1;
#pragma unroll
  for (int m = 0; m < 2; ++m) r.act[m] = m < ic.NL && r.s + r.lag[m] < D;
  return r;
}

__device__ __forceinline__ void fr_ic_put(const FrIc& ic, int64_t D, const FrIcRow& rw, int m, double nn, double icv,
                                          double ric, double beta) {
  double* o = ic.out + ((int64_t)(m * 4) * ic.F + rw.f) * D + rw.s + rw.lag[m];
  const int64_t stp = ic.F * D;
  o[0] = nn;
  o[stp] = icv;
  o[2 * stp] = ric;
  o[3 * stp] = beta;
}

// IC tail of k_cs_rank_fa<..., IC>: every thread calls it once the row's ranks are known,
// a barrier has retired every read of the bucketed keys and the row's exposures sit in LDS
// (xk[i]: the key registers are free again).  lds: the scratch after xk.  r2: the thread's
// doubled ranks among the row's non-NaN exposures (0: NaN), two per word; em: bit 2k+m set when element k is non-NaN and its lag-m return is NaN.  The
// pairs of lag m are the non-NaN exposures minus that list E_m; a pair's rank is r2 minus
// #(E_m < x) + #(E_m <= x), read off a 64-rank block table of E_m (as k_ic_wave).
// Moments: one pass of sums shifted by block-uniform anchors (xs: a sample key of the
// row, ic.rsh[t]: the target date's first non-NaN return), so wave partials simply add
// (records agree with the two-pass kernels to ~1e-15 relative, pair counts exactly).
// dynamic LDS of the IC variant: the row's exposures (A doubles), then the tail's E lists,
// block tables and wave partials
__host__ __device__ inline int64_t fr_ic_xk_words(int64_t A) { return (A * 8 + 15) / 16 * 4; }
__host__ __device__ inline int64_t fr_ic_lds_bytes(int64_t A, int nt) {
  const int64_t nbp = (((2 * A) >> 6) + 2) & ~1ll;
  return fr_ic_xk_words(A) * 4 + (2 * FR_IC_EC + 2 * nbp) * 4 + (int64_t)(nt / 64 + 1) * 20 * 8;
}

template <int EMAX>
__device__ __forceinline__ uint32_t fr_r2(const uint32_t* r2, int k) {
  return (r2[k / 2] >> (16 * (k % 2))) & 0xffffu;
}

template <int NT, int EMAX>
__device__ __forceinline__ void fr_ic_tail(const FrIc& ic, const FrIcRow& rw, int64_t D, int64_t A, int64_t ld,
                                           int64_t row, const double* xk, const uint32_t* r2, uint32_t em,
                                           bool last_in, double xs, uint32_t* lds, int* ne BR_PH_PARAMS) {
  constexpr int NW = NT / 64, S = 20;        // per-wave scratch: 2 lags x 8 sums, 2 x (count, flags)
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int nb = (int)((2 * A) >> 6) + 1;     // doubled ranks are <= 2A
  const int nbp = (nb + 1) & ~1;
  uint32_t* ebuf = lds;                       // [2][FR_IC_EC] E entries (unordered, then by block)
  uint32_t* T = lds + 2 * FR_IC_EC;           // [2][nbp] block table: start | end << 16
  double* scr = reinterpret_cast<double*>(lds + 2 * FR_IC_EC + 2 * nbp);
  // 1. unordered E lists
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      if ((em >> (2 * k + m)) & 1) {
        const int q = atomicAdd(&ne[m], 1);
        if (q < FR_IC_EC) ebuf[m * FR_IC_EC + q] = fr_r2<EMAX>(r2, k);
      }
    }
  }
  // lag 0's returns in flight over the table build
  (void)last_in;
  auto pair_of = [&](int k, int m) {           // non-NaN exposure (r2 > 0), non-NaN return
    return fr_in<NT>(t, k, (int)A) && fr_r2<EMAX>(r2, k) != 0u && !((em >> (2 * k + m)) & 1);
  };
  // unconditional loads (a branch per load serialises them): the last slot clamped into
  // the row, inactive lags read date s's row; non-pairs are skipped when summing
  auto load_r = [&](double* rv, const double* rr) {
#pragma unroll
    for (int k = 0; k < EMAX; ++k) rv[k] = rr[fr_ix<NT>(t, k, (int)A)];
  };
  double rv[EMAX];
  load_r(rv, ic.Rt + (rw.act[0] ? rw.s + rw.lag[0] : rw.s) * ld);
  BR_PH();
  __syncthreads();
  BR_PH();
  const int nE[2] = {ne[0], ne[1]};
  if ((rw.act[0] && nE[0] > FR_IC_EC) || (rw.act[1] && nE[1] > FR_IC_EC)) {
    // a long NaN-return list: k_ic_ranked_list takes the row from its doubled ranks
#pragma unroll
    for (int k = 0; k < EMAX; ++k)
      if (fr_in<NT>(t, k, (int)A)) ic.RK[row * ld + t + k * NT] = (fmx_rank2_t)fr_r2<EMAX>(r2, k);
    if (t == 0) {
      const int q = atomicAdd(&ic.ovf[0], 1);
      ic.ovf[1 + q] = (int32_t)fmx_blk();
    }
    return;
  }
  // 2. wave m counting-sorts lag m's entries into 64-rank blocks
  const bool wact = wid == 0 ? rw.act[0] : rw.act[1];   // (no dynamic register-array index)
  const int c = wid == 0 ? nE[0] : nE[1];
  if (wid < 2 && wact && c > 0) {
    uint32_t* Tm = T + wid * nbp;
    uint32_t* eb = ebuf + wid * FR_IC_EC;
    for (int b = lane; b < nbp; b += 64) Tm[b] = 0u;
    uint32_t er[FR_IC_EC / 64];
    int es[FR_IC_EC / 64];
#pragma unroll
    for (int q = 0; q < FR_IC_EC / 64; ++q) {
      const int j = 64 * q + lane;
      er[q] = j < c ? eb[j] : 0u;             // entries are doubled ranks >= 2
      es[q] = 0;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < FR_IC_EC / 64; ++q)
      if (er[q]) es[q] = (int)atomicAdd(&Tm[er[q] >> 6], 1u);
    __builtin_amdgcn_wave_barrier();
    const int R = (nbp + 63) >> 6;            // lane l owns blocks [l R, l R + R)
    int loc = 0;
    for (int q = 0; q < R; ++q) {
      const int b = lane * R + q;
      loc += b < nbp ? (int)Tm[b] : 0;
    }
    int incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = fr_up(incl, o, lane);
      if (lane >= o) incl += u;
    }
    int run = incl - loc;
    for (int q = 0; q < R; ++q) {
      const int b = lane * R + q;
      if (b < nbp) {
        const int n = (int)Tm[b];
        Tm[b] = (uint32_t)run | ((uint32_t)(run + n) << 16);
        run += n;
      }
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < FR_IC_EC / 64; ++q)
      if (er[q]) eb[(Tm[er[q] >> 6] & 0xffffu) + es[q]] = er[q];
  }
  BR_PH();
  __syncthreads();
  BR_PH();
  // 3. per lag: pair count (ballots), sums about the anchors (xs, ar), exact integer rank
  // sums; wave partials into scr
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    double a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int cnt = 0;
    uint32_t dif = 0;
    if (rw.act[m]) {                          // block-uniform
      const double* rr = ic.Rt + (rw.s + rw.lag[m]) * ld;
      if (m == 1) load_r(rv, rr);
      const double ar = ic.rsh[rw.s + rw.lag[m]];
      const uint32_t* Tm = T + m * nbp;
      const uint32_t* eb = ebuf + m * FR_IC_EC;
      const bool hasE = nE[m] > 0;
      uint64_t kk = 0;
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
        const bool pair = pair_of(k, m);
        cnt += __popcll(__ballot(pair));
        if (!pair) continue;
        const double x = xk[t + k * NT], r = rv[k];
        uint32_t k2 = fr_r2<EMAX>(r2, k);
        if (hasE) {
          const uint32_t tb = Tm[k2 >> 6];
          const uint32_t j0 = tb & 0xffffu, j1 = tb >> 16;
          uint32_t corr = 2u * j0;
          for (uint32_t j = j0; j < j1; ++j) {  // this block's entries (usually none)
            const uint32_t e = eb[j];
            corr += (e < k2 ? 1u : 0u) + (e <= k2 ? 1u : 0u);
          }
          k2 -= corr;
        }
        const double dx = x - xs, dy = r - ar;
        dif |= ((x != xs) ? 1u : 0u) | ((r != ar) ? 2u : 0u);
        a[0] += dx; a[1] += dy;
        a[2] += dx * dx; a[3] += dy * dy; a[4] += dx * dy;
        a[5] += (double)k2 * dy;
        kk += (uint64_t)k2 * k2;
      }
      a[7] = (double)kk;                      // a[6] unused (sum k = n(n+1) exactly)
    }
    fr_part_bfly<8, false>(a, scr, S, 8 * m);
    const uint32_t fl = (__ballot(dif & 1u) != 0 ? 1u : 0u) | (__ballot(dif & 2u) != 0 ? 2u : 0u);
    if (lane == 0) {
      scr[wid * S + 16 + 2 * m] = (double)cnt;
      scr[wid * S + 17 + 2 * m] = (double)fl;
    }
    BR_PH();
  }
  __syncthreads();
  BR_PH();
  // 4. wave 0: lane j < 20 totals value j over the waves (counts and sums add, flags OR);
  // lane 0 finishes both lags' records
  if (wid == 0) {
    double v = 0.0;
    uint32_t orf = 0;
    if (lane < S) {
      for (int w = 0; w < NW; ++w) {
        const double x = scr[w * S + lane];
        v += x;
        if (lane == 17 || lane == 19) orf |= (uint32_t)x;
      }
    }
    // totals through LDS (20 readlanes would hold 40 SGPRs and spill)
    double* tot = scr + NW * S;
    if (lane < S) tot[lane] = (lane == 17 || lane == 19) ? (double)orf : v;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane == 0) {
      const uint32_t fl0 = (uint32_t)tot[17], fl1 = (uint32_t)tot[19];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        if (!rw.act[m]) continue;
        const double* w = tot + 8 * m;
        const double n = tot[16 + 2 * m];
        const uint32_t fl = m == 0 ? fl0 : fl1;
        double icv = qnan(), ric = qnan(), beta = qnan();
        if (n >= 3.0) {
          const double s1 = w[0], s2 = w[1];
          if ((fl & 3u) == 3u) {              // neither side constant
            const double cxy = w[4] - s1 * s2 / n;
            const double cxx = w[2] - s1 * s1 / n;
            const double cyy = w[3] - s2 * s2 / n;
            // ranks: sum k = n(n+1)/2 (ties keep it), sum k^2 = sum (2k)^2 / 4: both exact
            const double ckk = w[7] / 4.0 - n * (n + 1.0) * (n + 1.0) / 4.0;
            const double cky = 0.5 * w[5] - 0.5 * (n + 1.0) * s2;
            icv = fmin(1.0, fmax(-1.0, cxy / sqrt(cxx * cyy)));
            ric = fmin(1.0, fmax(-1.0, cky / sqrt(ckk * cyy)));
          }
          // beta = sum x r / sum x^2 from the shifted sums
          const double a = xs, b = ic.rsh[rw.s + rw.lag[m]];
          const double sxx_raw = w[2] + 2.0 * a * s1 + n * a * a;
          const double sxr_raw = w[4] + a * s2 + b * s1 + n * a * b;
          beta = sxx_raw > 0 ? sxr_raw / sxx_raw : qnan();
        }
        fr_ic_put(ic, D, rw, m, n, icv, ric, beta);
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// cs_rank: y = (rank - 1) / (len(row) - 1), len counting NaN rows; 0.5 for single-row
// dates (operations.py:58-60).  Rows are (f, d) = blockIdx.x / D, % D.
//
// LDS is the occupancy limiter (rows in flight per CU hide each row's barrier and LDS
// latency chain), so the bucket counters and the bucketed keys share one buffer: the
// counters are read into registers after their scan, and only then are the keys of
// shared fine buckets scattered over them.  ~42 KB per row: three rows per CU.
// Positions t + k*NT with k < EMAX-1 are always inside the row (EMAX = ceil(A/NT)).
//
// WQ: also cs_winsor of the same row into Y2 (operations.py:64-68) from the same histogram.
// The four numpy 'linear' order statistics are read off the ranks: after the in-bucket
// scan every element knows #less / #equal among the valid keys, so the owner of order
// statistic k (less <= k < less + equal) publishes its key -- no second pass over the row.
//
// RK (optional): 2 * average rank among the row's valid keys, i.e. 2*#less + #equal + 1
// (0 for NaN / absent), as uint16 (<= 2A) -- the daily IC of the same rows starts from it
// (k_ic_wave) instead of ranking them again.
//
// IC (dense rows, method average): the daily IC records of the row's two lags from its
// ranks (fr_ic_tail) -- no doubled ranks written, no second pass over X.
//
// ZN (dense rows, with WQ): cs_zscore and market_neutralize of the same rows too -- the row is
// staged once in LDS (the region the counters take next) for numpy's pairwise nansum and
// sum of squared deviations (block_pw_sum_w0, bit-identical to k_cs_moment_rg), and the two
// outputs are written from it before the ranking starts: the row is read from HBM once for
// four operators (fmx_cs_rank_winsor_zn).
#ifndef FR_FA_LISTS
#define FR_FA_LISTS 0
#endif
template <int NT, int EMAX, bool PRES, bool WQ = false, bool IC = false, bool ZN = false, bool T64 = false>
__global__ void __launch_bounds__(NT, fr_fa_min_waves(NT, EMAX))
k_cs_rank_fa(const double* __restrict__ X, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld, int method,
             const uint8_t* __restrict__ present, double* __restrict__ Y2, double qlo, double qhi,
             fmx_rank2_t* __restrict__ RK, FrIc ic, FrZn zn, int lcap) {
  constexpr int K = FR_K_CS, NW = NT / 64;
  constexpr int WORDS = FR_CS_WORDS, DUMMY = 2 * WORDS - 1;   // sentinel bucket: last half-word
  static_assert(FRG<K>::NB + 1 < DUMMY, "counter array");
  __shared__ FrTab tab;
  __shared__ uint4 wred[NW];                  // per wave: #present, #valid, min / max key high words
  __shared__ int iscr[NW];
  // dynamic: max(A keys, WORDS packed counters), then the scan list (lcap items; with ZN the
  // moments' schedule and tree nodes alias it)
  extern __shared__ uint64_t lds[];
  uint32_t* cnt = (uint32_t*)lds;             // 16-bit counter of bucket b: half b & 1 of word b >> 1
  uint64_t* bkey = lds;
  uint32_t* litems = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(lds) + fr_list_off(A, WORDS));
  const int t = threadIdx.x, wid = t >> 6;
  BR_PH_INIT;
  static_assert(!(IC && PRES), "the fused IC ranks dense rows");
  static_assert(!ZN || (WQ && !PRES && !IC), "ZN: dense rank + winsor rows");
  static_assert(!T64 || (ZN && NT == 512), "T64: the fused pass's 64-leaf moment trees");
  int32_t* zn_sch = reinterpret_cast<int32_t*>(litems);
  double* zn_nodes = reinterpret_cast<double*>(litems + PW_LDS_MAX);
  __shared__ int zn_iscr[ZN ? NW + 2 : 1];
  FrIcRow rw{};
  __shared__ int ic_ne[2];                    // E-list lengths (IC)
  if constexpr (IC) {
    rw = fr_ic_row(ic, D);
    if (t < 2) ic_ne[t] = 0;
  }
  // grid dim3(dates, F): row (f, d) = f * D + x, the panel pointers offset by the range's
  // first date (a date sub-range: the sharded step's owned dates, fmx_*_dates)
  const int64_t row = IC ? rw.f * D + rw.s : (int64_t)blockIdx.y * D + blockIdx.x;
  const double* x = X + row * ld;
  double* y = Y + row * ld;
  const uint8_t* prow = PRES ? present + (row % D) * ld : nullptr;
  const int An = (int)A;
  const bool last_in = t + (EMAX - 1) * NT < An;
  uint64_t key[EMAX];
  uint32_t pm = 0, hmin = 0xffffffffu, hmax = 0u;
  int wv = 0, wp = 0;                         // wave-uniform counts (ballots)
  // every load of the row issued before the first is consumed: a load under a branch (the
  // key conversion below is one per element) waits out the previous one's HBM latency.
  // The last slot is clamped into the row (its value is unused when out of range).
  double xv[EMAX];
  uint32_t pv = 0;
#pragma unroll
  for (int k = 0; k < EMAX; ++k) xv[k] = x[fr_ix<NT>(fr_opaque(t), k, (int)A)];
  if (PRES) {
#pragma unroll
    for (int k = 0; k < EMAX; ++k) pv |= (prow[fr_ix<NT>(t, k, (int)A)] != 0 ? 1u : 0u) << k;
  }
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const bool in = fr_in<NT>(t, k, (int)A);
    const double v = xv[k];
    const bool p = in && (PRES ? ((pv >> k) & 1u) != 0 : true);
    const bool ok = p && v == v;
    pm |= (uint32_t)p << k;
    key[k] = ok ? okey(v) : KEY_SENTINEL;
    const uint32_t h = (uint32_t)(key[k] >> 32);
    hmin = ok ? min(hmin, h) : hmin;
    hmax = ok ? max(hmax, h) : hmax;
    wv += __popcll(__ballot(ok));
    if (PRES) wp += __popcll(__ballot(p));
    if constexpr (ZN)
      if (in) reinterpret_cast<double*>(lds)[fr_opaque(t) + k * NT] = v;   // the row for the moments
  }
  BR_PH();
  if constexpr (ZN) {
    // cs_zscore / market_neutralize: numpy nanmean and nanvar (ddof 0) by the pairwise
    // schedule of n = A (NaN -> 0 in the sums, counted apart), as k_cs_moment_rg
    const double* vrow = reinterpret_cast<const double*>(lds);
    const int32_t* g = zn.pw.get(An);
    const bool sl = zn.slen <= PW_LDS_MAX;
    if (sl)
      for (int i = t; i < zn.slen; i += NT) zn_sch[i] = g[i];
    // the rank phase's sample and row bounds now, so that wave 1 builds the splitter table
    // while wave 0 combines the first moment sum (no serial table phase of its own)
    fr_park_sample<NT, EMAX>(tab, key);
    {
      const uint32_t a = fr_wave_min_u32(hmin), c = fr_wave_max_u32(hmax);
      if ((t & 63) == 0) wred[wid] = make_uint4((uint32_t)wp, (uint32_t)wv, a, c);
    }
    __syncthreads();
    const int32_t* sch = sl ? zn_sch : g;
    auto table = [&]() {
      int nv1 = 0;
      uint32_t a0 = 0xffffffffu, a1 = 0u;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        const uint4 r = wred[w];
        nv1 += (int)r.y;
        a0 = min(a0, r.z);
        a1 = max(a1, r.w);
      }
      if (nv1 > 0 && An > 1) {                // the rows that rank (dense, method average)
        double vmin, vmax;
        fr_key_bounds(a0, a1, &vmin, &vmax);
        fr_build_w0<K>(tab, FR_FROM_LDS, vmin, vmax);
      }
    };
#ifdef FR_DIAG_NOZNSUM
    int cnt = An; (void)sch; table();
    const double s1 = vrow[t], mean = s1, s2 = vrow[t + 1], var = s2;
#else
    // the non-NaN count is the rank phase's #valid keys (its ballots, in wred since the
    // barrier above): no per-element count in the moment leaves
    int c1, c2, cnt = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) cnt += (int)wred[w].y;
    auto e1 = [&](int i) { const double u = vrow[i]; return u == u ? u : 0.0; };
    double s1, s2;
    // T64: the row length's tree is complete over 64 leaves (the launcher checks pw_tree64)
    if constexpr (T64) s1 = block_pw_sum_t64<NT>(e1, sch, zn_nodes, table);
    else s1 = block_pw_sum_w0<NT>(e1, [](int) { return 0; }, sch, zn_nodes, zn_iscr, &c1, table);
    const double mean = cnt > 0 ? s1 / (double)cnt : qnan();
    BR_PH();
    // (mean - u)^2 for a valid u, 0 for NaN: numpy's (mean - where(nan, 0, u))^2 masked to 0
    auto e2 = [&](int i) {
      const double u = vrow[i];
      return u == u ? (mean - u) * (mean - u) : 0.0;
    };
    if constexpr (T64) s2 = block_pw_sum_t64<NT>(e2, sch, zn_nodes + 8);
    else s2 = block_pw_sum_w0<NT>(e2, [](int) { return 0; }, sch, zn_nodes, zn_iscr, &c2);
    const double var = cnt > 0 ? s2 / (double)cnt : qnan();
#endif
    BR_PH();
    const double sd = sqrt(var);
    const bool g2 = sd == 0.0 || sd != sd;     // neutralize: sigma in {0, NaN} -> 0
    const double rsd = 1.0 / sd;               // (x - mean) / sd by rdiv: bit-identical
    const bool sd_ok = rdiv_ok(sd);
    double* yz = zn.Yz + row * ld;
    double* yn = zn.Yn + row * ld;
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (!fr_in<NT>(t, k, (int)A)) continue;
      const int ia = fr_opaque(t) + k * NT;
      const double o = rdiv(vrow[ia] - mean, sd, rsd, sd_ok);
      __builtin_nontemporal_store(o, yz + ia);
      __builtin_nontemporal_store(g2 ? 0.0 : o, yn + ia);
    }
    __syncthreads();                          // every read of the staged row is done
    BR_PH();
  }
  if constexpr (!ZN) fr_park_sample<NT, EMAX>(tab, key);
#pragma unroll
  for (int j = 0; j < WORDS / (4 * NT); ++j)
    reinterpret_cast<uint4*>(cnt)[t * (WORDS / (4 * NT)) + j] = make_uint4(0u, 0u, 0u, 0u);
  if constexpr (!ZN) {
    const uint32_t a = fr_wave_min_u32(hmin), c = fr_wave_max_u32(hmax);
    if ((t & 63) == 0) wred[wid] = make_uint4((uint32_t)wp, (uint32_t)wv, a, c);
  }
  __syncthreads();
  BR_PH();
  int nrow = An, nv = 0;
  uint32_t h0 = 0xffffffffu, h1 = 0u;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const uint4 r = wred[w];
    if (PRES) nrow = (w == 0 ? 0 : nrow) + (int)r.x;
    nv += (int)r.y;
    h0 = min(h0, r.z);
    h1 = max(h1, r.w);
  }
  if ((method == FMX_RANK_AVERAGE_PROPAGATE && nv < nrow) || nv == 0 ||
      (method != FMX_RANK_AVERAGE_PROPAGATE && nrow == 1)) {
    // scipy propagate: one NaN -> all NaN; single-row date -> 0.5 (operations.py:58)
    const bool half = (method != FMX_RANK_AVERAGE_PROPAGATE) && nrow == 1;
    if (Y) {                                  // Y == NULL: doubled ranks only (fmx_cs_rank2)
#pragma unroll
      for (int k = 0; k < EMAX; ++k)
        if (fr_in<NT>(t, k, (int)A)) y[fr_opaque(t) + k * NT] = (((pm >> k) & 1) && half) ? 0.5 : qnan();
    }
    if (RK) {                                 // nv == 0 or a single-row date (rank 1)
#pragma unroll
      for (int k = 0; k < EMAX; ++k)
        if (fr_in<NT>(t, k, (int)A)) RK[row * ld + fr_opaque(t) + k * NT] = (fmx_rank2_t)(key[k] == KEY_SENTINEL ? 0u : 2u);
    }
    if (WQ) {                                 // nv < 5: winsor is the identity
#pragma unroll
      for (int k = 0; k < EMAX; ++k)
        if (fr_in<NT>(t, k, (int)A)) Y2[row * ld + fr_opaque(t) + k * NT] = key[k] == KEY_SENTINEL ? qnan() : okey_inv(key[k]);
    }
    if constexpr (IC) {                       // < 3 pairs: empty records (n = 0, or 1 on a one-asset row)
      if (t == 0) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          if (!rw.act[m]) continue;
          const double r = ic.Rt[(rw.s + rw.lag[m]) * ld];
          const double n = (nv > 0 && key[0] != KEY_SENTINEL && r == r) ? 1.0 : 0.0;
          fr_ic_put(ic, D, rw, m, n, qnan(), qnan(), qnan());
        }
      }
    }
    return;
  }
  if (!ZN && wid == 0) {                      // (ZN: wave 1 built it during the moments)
    double vmin, vmax;
    fr_key_bounds(h0, h1, &vmin, &vmax);
    fr_build_w0<K>(tab, FR_FROM_LDS, vmin, vmax);
  }
  if constexpr (!ZN) __syncthreads();         // (ZN: the counters' zeroing barrier covers it)
  BR_PH();
  int sl[EMAX];                               // slot | bucket << PK_BSHIFT, then start | len << 16
  {
    int bb[EMAX];
    fr_bucket_all<K, EMAX, (NT >= 1024 ? 2 : 4), true>(tab, key, bb, DUMMY);
#pragma unroll
    for (int k = 0; k < EMAX; ++k) sl[k] = (int)fr_cnt_add(cnt, bb[k] & (FR_BEQ - 1)) | (bb[k] << PK_BSHIFT);
  }
  __syncthreads();
  BR_PH();
  fr_scan16<NT, WORDS>(cnt, iscr);
  BR_PH();
  // le[k] = #less | #equal << 16 inside the bucket; for elements still to scan (n field of
  // sl set) first their work item in the wave's list region (fr_claim_put).  Per-wave work
  // lists for long rows and the winsor passes, per-slot loops for short rank-only rows
  // (measured per 252 dates: A = 5000 cs_rank 1.60 vs 1.68 ms, cs_rank_winsor 2.13 vs 2.30
  // with lists; A = 3000 cs_rank 9.42 vs 10.13 ms and the C4 rank pass 9.38 vs 10.04 with
  // per-slot loops, its cs_rank_winsor 12.11 vs 12.29 with lists).  FR_FA_LISTS=1: lists
  // everywhere (A/B)
  int le[EMAX];
  if constexpr (ZN || WQ || EMAX >= 8 || FR_FA_LISTS) {
    const int wcap = lcap / NW;
    uint32_t* witems = litems + wid * wcap;
    FrClaim lcl;
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const int b = (sl[k] >> PK_BSHIFT) & (FR_BEQ - 1);
      const int slot = sl[k] & PK_SLOT;
      int s0, s1;
      fr_cnt_get2(cnt, b, &s0, &s1);
      const int n = s1 - s0;
      const bool eqb = (sl[k] >> PK_BSHIFT) & FR_BEQ;   // equal-to-sample bucket: all members tie
      const bool scan = !eqb && n > 1 && b != DUMMY;
      const int ref = fr_claim_put(lcl, witems, wcap, scan, n, slot, s0);
      le[k] = scan ? ref : (eqb ? n : 1) << 16;
      sl[k] = s0 | (scan ? n << 16 : 0);
      FR_SCHED_FENCE();
    }
    __syncthreads();                          // counters dead: the keys reuse their LDS
    BR_PH();
#pragma unroll
    for (int k = 0; k < EMAX; ++k)
      if (sl[k] >> 16) fr_scatter_key(bkey, le[k], sl[k] & 0xffff, key[k]);
    __syncthreads();
    BR_PH();
#ifndef FR_DIAG_NOSCAN
    fr_list_walk_wave(bkey, witems, wcap, lcl);
#endif
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const int n = sl[k] >> 16;
      if (n) le[k] = fr_result(bkey, witems, le[k], sl[k] & 0xffff, n);
    }
    BR_PH();
  } else {
    (void)lcap;
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const int b = (sl[k] >> PK_BSHIFT) & (FR_BEQ - 1);
      const int slot = sl[k] & PK_SLOT;
      int s0, s1;
      fr_cnt_get2(cnt, b, &s0, &s1);
      const int n = s1 - s0;
      const bool eqb = (sl[k] >> PK_BSHIFT) & FR_BEQ;   // equal-to-sample bucket: all members tie
      const bool scan = !eqb && n > 1 && b != DUMMY;
      le[k] = scan ? slot : (eqb ? n : 1) << 16;
      sl[k] = s0 | (scan ? n << 16 : 0);
    }
    __syncthreads();                          // counters dead: the keys reuse their LDS
    BR_PH();
#pragma unroll
    for (int k = 0; k < EMAX; ++k)
      if (sl[k] >> 16) bkey[(sl[k] & 0xffff) + le[k]] = key[k];
    __syncthreads();
    BR_PH();
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const int n = sl[k] >> 16;
      if (n) {
        const uint64_t* bk = bkey + (sl[k] & 0xffff);
        const uint64_t own = bk[le[k]];       // own key from its slot: keys dead after the scatter
        int lt = 0, eq = 0;
#pragma unroll 2
        for (int j = 0; j < n; ++j) {
          const uint64_t w = bk[j];
          lt += w < own ? 1 : 0;
          eq += w == own ? 1 : 0;
        }
        le[k] = lt | eq << 16;
      }
    }
    BR_PH();
  }
  const double den = (double)(nrow - 1);
  const double rden = 1.0 / den;              // (r - 1) / den through mdiv: bit-identical
  // winsor order statistics (numpy linear) of the nv valid keys
  __shared__ uint64_t tval[4];
  int kk[4] = {0, 0, 0, 0};
  double gq[2] = {0.0, 0.0};
  if (WQ && nv >= 5) {
    const double qs[2] = {qlo, qhi};
#pragma unroll
    for (int z = 0; z < 2; ++z) {
      const double vi = (double)(nv - 1) * qs[z];
      if (vi >= (double)(nv - 1)) {
        kk[2 * z] = kk[2 * z + 1] = nv - 1;
        gq[z] = vi + 1.0;
      } else {
        const double pf = floor(vi);
        kk[2 * z] = (int)pf;
        kk[2 * z + 1] = (int)pf + 1;
        gq[z] = vi - pf;
      }
    }
  }
  uint32_t r2[IC ? (EMAX + 1) / 2 : 1];       // IC: doubled ranks (0: NaN), two 16-bit per word
  uint32_t em = 0;                            // IC: bit 2k+m = non-NaN exposure, NaN lag-m return
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    if constexpr (IC) if (k % 2 == 0) r2[k / 2] = 0u;
    if (!fr_in<NT>(t, k, (int)A)) continue;
    const int lt = le[k] & 0xffff, eq = le[k] >> 16;
    const int less = (sl[k] & 0xffff) + lt;
    if constexpr (IC) r2[k / 2] |= (key[k] != KEY_SENTINEL ? (uint32_t)(2 * less + eq + 1) : 0u) << (16 * (k % 2));
    // write-once outputs: nontemporal stores
    const int ia = fr_opaque(t) + k * NT;       // recomputed here, not kept from the loads
    if constexpr (ZN) {
      // method average: (r - 1) / den with r = r2 / 2, r2 = 2 less + eq + 1 the doubled rank;
      // (r2 - 2) / (2 den) is the same real number (r - 1 = (r2 - 2) / 2 exactly), so
      // mdiv(r2 - 2, 2 den, RN(1 / den) / 2) gives the same bits from one conversion
      const double q = mdiv((double)(2 * less + eq - 1), 2.0 * den, 0.5 * rden);
      __builtin_nontemporal_store(key[k] == KEY_SENTINEL ? qnan() : q, y + ia);
    } else {
      double r;
      if (method == FMX_RANK_MIN) r = (double)(less + 1);
      else if (method == FMX_RANK_MAX) r = (double)(less + eq);
      else r = (double)less + (double)(eq + 1) / 2.0;
      if (Y) __builtin_nontemporal_store(key[k] == KEY_SENTINEL ? qnan() : mdiv(r - 1.0, den, rden), y + ia);
    }
    if (RK) __builtin_nontemporal_store((fmx_rank2_t)(key[k] == KEY_SENTINEL ? 0u : (uint32_t)(2 * less + eq + 1)),
                                        RK + row * ld + ia);
    if (WQ && nv >= 5) {
      // the owners of the four order statistics (less <= kk < less + eq) publish their key;
      // four hits per row, so the divergent stores sit behind a wave-uniform test
      uint32_t hm = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) hm |= ((uint32_t)(kk[j] - less) < (uint32_t)eq ? 1u : 0u) << j;
      if (key[k] == KEY_SENTINEL) hm = 0;
      if (__builtin_amdgcn_ballot_w64(hm != 0)) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if ((hm >> j) & 1u) tval[j] = key[k];   // all writers store the same key
      }
    }
  }
  if constexpr (IC) {
    // E membership: non-NaN exposure whose lag-m return is NaN (bit rows of k_nan_bits)
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      if (!rw.act[m]) continue;
      const uint32_t* nb = ic.nanb + (rw.s + rw.lag[m]) * ic.nw;
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
        const int i = fr_in<NT>(t, k, (int)A) ? t + k * NT : 0;   // unconditional loads
        const uint32_t bit = (nb[i >> 5] >> (i & 31)) & 1u;
        if (fr_in<NT>(t, k, (int)A) && key[k] != KEY_SENTINEL) em |= bit << (2 * k + m);
      }
    }
  }
  if (WQ) {
    __syncthreads();
    double lo = qnan(), hi = qnan();
    if (nv >= 5) {
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
    double* y2 = Y2 + row * ld;
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (!fr_in<NT>(t, k, (int)A)) continue;
      const double v = key[k] == KEY_SENTINEL ? qnan() : okey_inv(key[k]);
      double o = v;
      if (nv >= 5) o = (v < lo) ? lo : ((v > hi) ? hi : v);
      __builtin_nontemporal_store((PRES && !((pm >> k) & 1)) ? qnan() : o, y2 + fr_opaque(t) + k * NT);
    }
  }
  if constexpr (IC) {
    if constexpr (!WQ) __syncthreads();       // (WQ: its barrier) every in-bucket scan read is done
    // the exposures move to LDS (read once per lag by their owner): frees the key registers
    double* xk = reinterpret_cast<double*>(lds);
#pragma unroll
    for (int k = 0; k < EMAX; ++k)
      if (fr_in<NT>(t, k, (int)A)) xk[t + k * NT] = key[k] != KEY_SENTINEL ? okey_inv(key[k]) : 0.0;
    // exposure anchor: a sample key of the row (block-uniform, the sorted samples in tab)
    const uint64_t sk = tab.spl[31] != KEY_SENTINEL ? tab.spl[31] : tab.spl[0];
    const double xs = sk != KEY_SENTINEL ? okey_inv(sk) : 0.0;
    BR_PH();
    fr_ic_tail<NT, EMAX>(ic, rw, D, A, ld, row, xk, r2, em, last_in, xs,
                         reinterpret_cast<uint32_t*>(lds) + fr_ic_xk_words(A), ic_ne BR_PH_ARGS);
  }
  BR_PH();
}

// Bucket ids of a thread's keys, group by group (fr_bucket_grp), each group's LDS counter
// increments issued right away: sl[k] = slot | bucket << PK_BSHIFT.  The scheduling fence
// keeps the compiler from interleaving every group's searches and final selects (all EMAX
// sample words in flight at once).
template <int K, int EMAX, int G>
__device__ __forceinline__ void fr_bucket_cnt(const FrTab& T, const uint64_t* key, int* sl, int dummy,
                                              uint32_t* cnt) {
  constexpr int g = EMAX < G ? EMAX : G;
  int b[g];
  fr_bucket_grp<K, g, true>(T, key, b, dummy);
#pragma unroll
  for (int k = 0; k < g; ++k) sl[k] = (int)fr_cnt_add(cnt, b[k] & (FR_BEQ - 1)) | (b[k] << PK_BSHIFT);
  FR_SCHED_FENCE();
  if constexpr (EMAX > G) fr_bucket_cnt<K, EMAX - G, G>(T, key + G, sl + G, dummy, cnt);
}

// ------------------------------------------------------------------------------------
// Doubled average ranks only, persistent (fmx_cs_rank2 on rows of 8193..16384 assets: the
// rank pass in front of a daily IC over a panel no operator ranks, e.g. C5's feature panel).
// One 1024-thread workgroup per CU walks rows b, b + G, ...; the next row's loads are issued
// as soon as the current row's keys are formed and land during its bucket phases (its HBM
// latency was the exposed third of a row's time).  At one row per CU the kernel has 128
// VGPRs: keys, the prefetched row and the per-element state fit without spills (two rows
// per CU at 64 VGPRs spilled the keys).  Bucket pipeline and per-element results as
// k_cs_rank_fa (dense, method average, RK only):
//   rank2 = 2 * #less + #equal + 1 (0 for NaN); single-asset rows -> 2.
#ifndef FR_PF_LISTS
#define FR_PF_LISTS 0
#endif
template <int NT, int EMAX>
__global__ void __launch_bounds__(NT, 4)
k_cs_rank2_pf(const double* __restrict__ X, int64_t nrows, int64_t A, int64_t ld, fmx_rank2_t* __restrict__ RK,
              int lcap) {
  constexpr int K = FR_K_CS, NW = NT / 64;
  constexpr int WORDS = FR_CS_WORDS, DUMMY = 2 * WORDS - 1;
  static_assert(FRG<K>::NB + 1 < DUMMY, "counter array");
  __shared__ FrTab tab;
  __shared__ uint4 wred[NW];
  __shared__ int iscr[NW];
  extern __shared__ uint64_t lds[];           // max(A keys, WORDS packed counters), then the scan list
  uint32_t* cnt = (uint32_t*)lds;
  uint64_t* bkey = lds;
  uint32_t* litems = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(lds) + fr_list_off(A, WORDS));
  const int t = threadIdx.x, wid = t >> 6;
  const int An = (int)A;
  BR_PH_INIT;
  double xv[EMAX];
  int64_t row = blockIdx.x;
  if (row >= nrows) return;
#pragma unroll
  for (int k = 0; k < EMAX; ++k) xv[k] = X[row * ld + (fr_ix<NT>(fr_opaque(t), k, (int)A))];
  for (; row < nrows; row += gridDim.x) {
    BR_PH_ROW();
    uint64_t key[EMAX];
    uint32_t hmin = 0xffffffffu, hmax = 0u;
    int wv = 0;
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const double v = xv[k];
      const bool ok = fr_in<NT>(t, k, (int)A) && v == v;
      key[k] = ok ? okey(v) : KEY_SENTINEL;
      const uint32_t h = (uint32_t)(key[k] >> 32);
      hmin = ok ? min(hmin, h) : hmin;
      hmax = ok ? max(hmax, h) : hmax;
      wv += __popcll(__ballot(ok));
    }
    {                                         // the next row's loads (clamped to the last row)
#ifdef FR_DIAG_NOPF
      const int64_t nxt = row;
#else
      const int64_t nxt = row + gridDim.x < nrows ? row + gridDim.x : row;
#endif
#pragma unroll
      for (int k = 0; k < EMAX; ++k) xv[k] = X[nxt * ld + (fr_ix<NT>(fr_opaque(t), k, (int)A))];
    }
    fr_park_sample<NT, EMAX>(tab, key);
    BR_PH();
    __syncthreads();                          // the previous row's scan reads of bkey are done
    BR_PH();
  #pragma unroll
    for (int j = 0; j < WORDS / (4 * NT); ++j)
      reinterpret_cast<uint4*>(cnt)[t * (WORDS / (4 * NT)) + j] = make_uint4(0u, 0u, 0u, 0u);
    {
      const uint32_t a = fr_wave_min_u32(hmin), c = fr_wave_max_u32(hmax);
      if ((t & 63) == 0) wred[wid] = make_uint4(0u, (uint32_t)wv, a, c);
    }
    __syncthreads();
    BR_PH();
    int nv = 0;
    uint32_t h0 = 0xffffffffu, h1 = 0u;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint4 r = wred[w];
      nv += (int)r.y;
      h0 = min(h0, r.z);
      h1 = max(h1, r.w);
    }
    fmx_rank2_t* rk = RK + row * ld;
    if (nv == 0 || An == 1) {                 // no valid key / a single-asset row (rank 1)
#pragma unroll
      for (int k = 0; k < EMAX; ++k)
        if (fr_in<NT>(t, k, (int)A)) rk[fr_opaque(t) + k * NT] = (fmx_rank2_t)(key[k] == KEY_SENTINEL ? 0u : 2u);
      continue;                               // block-uniform
    }
    if (wid == 0) {
      double vmin, vmax;
      fr_key_bounds(h0, h1, &vmin, &vmax);
      
      fr_build_w0<K>(tab, FR_FROM_LDS, vmin, vmax);
    }
    __syncthreads();
    BR_PH();
    int sl[EMAX];
    
    fr_bucket_cnt<K, EMAX, 4>(tab, key, sl, DUMMY, cnt);
    __syncthreads();
    BR_PH();
    fr_scan16<NT, WORDS>(cnt, iscr);
    BR_PH();
#if FR_PF_LISTS
    int le[EMAX];                             // work item / slot, then c = 2 #less + #equal in the bucket
    uint32_t nan_m = 0;
    const int wcap = lcap / NW;
    uint32_t* witems = litems + wid * wcap;
    FrClaim lcl;
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const int b = (sl[k] >> PK_BSHIFT) & (FR_BEQ - 1);
      const int slot = sl[k] & PK_SLOT;
      int s0, s1;
      fr_cnt_get2(cnt, b, &s0, &s1);
      const int n = s1 - s0;
      const bool eqb = (sl[k] >> PK_BSHIFT) & FR_BEQ;   // equal-to-sample bucket: all members tie
      const bool scan = !eqb && n > 1 && b != DUMMY;
      nan_m |= (uint32_t)(b == DUMMY) << k;
      const int ref = fr_claim_put(lcl, witems, wcap, scan, n, slot, s0);
      le[k] = scan ? ref : (eqb ? n : 1);
      sl[k] = s0 | (scan ? n << 16 : 0);
      FR_SCHED_FENCE();
    }
    __syncthreads();                          // counters dead: the keys reuse their LDS
    BR_PH();
#pragma unroll
    for (int k = 0; k < EMAX; ++k)
      if (sl[k] >> 16) fr_scatter_key(bkey, le[k], sl[k] & 0xffff, key[k]);
    __syncthreads();
    BR_PH();
#ifndef FR_DIAG_NOSCAN
    fr_list_walk_wave(bkey, witems, wcap, lcl);
#endif
    BR_PH();
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const int n = sl[k] >> 16;
      if (n) {
        const int c = fr_result(bkey, witems, le[k], sl[k] & 0xffff, n);
        le[k] = 2 * (c & 0xffff) + (c >> 16);
      }
    }
#else
    // in-bucket scans as per-slot loops (each element walks its own bucket): at one 1024-thread
    // row per CU the per-wave work lists of k_cs_rank_fa cost more than they balance
    // (C5 rank pass 115.5 vs 104.3 ms)
    int le[EMAX];                             // scatter slot, then c = 2 #less + #equal in the bucket
    uint32_t nan_m = 0;
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const int b = (sl[k] >> PK_BSHIFT) & (FR_BEQ - 1);
      const int slot = sl[k] & PK_SLOT;
      int s0, s1;
      fr_cnt_get2(cnt, b, &s0, &s1);
      const int n = s1 - s0;
      const bool eqb = (sl[k] >> PK_BSHIFT) & FR_BEQ;   // equal-to-sample bucket: all members tie
      const bool scan = !eqb && n > 1 && b != DUMMY;
      nan_m |= (uint32_t)(b == DUMMY) << k;
      le[k] = scan ? slot : (eqb ? n : 1);
      sl[k] = s0 | (scan ? n << 16 : 0);
    }
    __syncthreads();                          // counters dead: the keys reuse their LDS
    BR_PH();
#pragma unroll
    for (int k = 0; k < EMAX; ++k)
      if (sl[k] >> 16) bkey[(sl[k] & 0xffff) + le[k]] = key[k];
    __syncthreads();
    BR_PH();
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const int n = sl[k] >> 16;
      if (n) {
        const uint64_t* bk = bkey + (sl[k] & 0xffff);
        const uint64_t own = bk[le[k]];       // own key from its slot: keys dead after the scatter
        int c = 0;
#pragma unroll 2
        for (int j = 0; j < n; ++j) {
          const uint64_t w = bk[j];
          c += (w < own ? 2 : 0) + (w == own ? 1 : 0);
        }
        le[k] = c;
      }
    }
    BR_PH();
#endif
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (!fr_in<NT>(t, k, (int)A)) continue;
      const uint32_t r2 = ((nan_m >> k) & 1u) ? 0u : (uint32_t)(2 * (sl[k] & 0xffff) + le[k] + 1);
#ifdef FR_DIAG_NOSTORE
      if (r2 == 0xfffffu)
#endif
      __builtin_nontemporal_store((fmx_rank2_t)r2, rk + fr_opaque(t) + k * NT);
    }
    BR_PH();
  }
}

// ------------------------------------------------------------------------------------
// cs_winsor (OP 0: clip to the quantiles when >= 5 non-NaN) / cs_filter_center (OP 1)
// on fine buckets (operations.py:64-75).  The numpy 'linear' percentiles need four order
// statistics; the fine-bucket histogram (one LDS atomic per element, one scan) locates
// the bucket of each, and only the members of those (tiny) buckets are gathered and
// ranked -- no per-element rank.  A bucket holding more than FR_QCAP members (heavily
// clustered rows) falls back to a bisection of the key space with block counts.
// LDS: the counters (32 KB) are dead once the four target buckets are known, and the
// gathered lists reuse them: four rows per CU at 512 threads.
constexpr int FR_QCAP = 1024;
template <int OP, int NT, int EMAX, bool PRES>
#ifndef FR_Q_WAVES
#define FR_Q_WAVES 6
#endif
__global__ void __launch_bounds__(NT, FR_Q_WAVES)
k_cs_quantile_fa(const double* __restrict__ X, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld,
                 double qlo, double qhi, const uint8_t* __restrict__ present) {
  constexpr int K = FR_K_CS, NW = NT / 64, NB = FRG<K>::NB;
  constexpr int WORDS = FR_CS_WORDS, DUMMY = 2 * WORDS - 1;
  static_assert(NB + 1 < DUMMY, "counter array");
  static_assert(4 * FR_QCAP * 2 <= WORDS, "lists alias the counters");
  __shared__ FrTab tab;
  __shared__ uint4 wred[NW];
  __shared__ int iscr[2 * (NW + 1)];
  __shared__ int tfill[4];
  __shared__ uint64_t tval[4];
  extern __shared__ uint64_t lds[];           // WORDS packed counters, then 4 lists of keys
  uint32_t* cnt = (uint32_t*)lds;
  uint64_t* lists = lds;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int64_t row = fmx_blk();              // grid dim3(D, F)
  const double* x = X + row * ld;
  double* y = Y + row * ld;
  const uint8_t* prow = PRES ? present + (row % D) * ld : nullptr;
  uint64_t key[EMAX];
  uint32_t pm = 0, hmin = 0xffffffffu, hmax = 0u;
  int wv = 0;
  // all loads in flight before the first is consumed (as k_cs_rank_fa)
  double xv[EMAX];
  uint32_t pv = 0;
#pragma unroll
  for (int k = 0; k < EMAX; ++k) xv[k] = x[fr_ix<NT>(t, k, (int)A)];
  if (PRES) {
#pragma unroll
    for (int k = 0; k < EMAX; ++k) pv |= (prow[fr_ix<NT>(t, k, (int)A)] != 0 ? 1u : 0u) << k;
  }
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const bool in = fr_in<NT>(t, k, (int)A);
    const double v = xv[k];
    const bool p = in && (PRES ? ((pv >> k) & 1u) != 0 : true);
    const bool ok = p && v == v;
    pm |= (uint32_t)p << k;
    key[k] = ok ? okey(v) : KEY_SENTINEL;
    const uint32_t h = (uint32_t)(key[k] >> 32);
    hmin = ok ? min(hmin, h) : hmin;
    hmax = ok ? max(hmax, h) : hmax;
    wv += __popcll(__ballot(ok));
  }
  fr_park_sample<NT, EMAX>(tab, key);
#pragma unroll
  for (int j = 0; j < WORDS / (4 * NT); ++j)
    reinterpret_cast<uint4*>(cnt)[t * (WORDS / (4 * NT)) + j] = make_uint4(0u, 0u, 0u, 0u);
  if (t < 4) tfill[t] = 0;
  {
    const uint32_t a = fr_wave_min_u32(hmin), c = fr_wave_max_u32(hmax);
    if (lane == 0) wred[wid] = make_uint4(0u, (uint32_t)wv, a, c);
  }
  __syncthreads();
  int nv = 0;
  uint32_t h0 = 0xffffffffu, h1 = 0u;
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const uint4 r = wred[w];
    nv += (int)r.y;
    h0 = min(h0, r.z);
    h1 = max(h1, r.w);
  }
  double lo = qnan(), hi = qnan();
  if (nv > 0 && (OP == 1 || nv >= 5)) {
    if (wid == 0) {
      double vmin, vmax;
      fr_key_bounds(h0, h1, &vmin, &vmax);
      fr_build_w0<K>(tab, FR_FROM_LDS, vmin, vmax);
    }
    __syncthreads();
    int bb[EMAX];
    fr_bucket_all<K, EMAX>(tab, key, bb, DUMMY);
#pragma unroll
    for (int k = 0; k < EMAX; ++k) fr_cnt_add(cnt, bb[k]);
    __syncthreads();
    fr_scan16<NT, WORDS>(cnt, iscr);
    // order statistics (p, p+1) per quantile (numpy linear), identical when vi >= n-1
    const double qs[2] = {qlo, qhi};
    double gq[2];
    int kk[4];
#pragma unroll
    for (int z = 0; z < 2; ++z) {
      const double vi = (double)(nv - 1) * qs[z];
      if (vi >= (double)(nv - 1)) {
        kk[2 * z] = kk[2 * z + 1] = nv - 1;
        gq[z] = vi + 1.0;
      } else {
        const double pf = floor(vi);
        kk[2 * z] = (int)pf;
        kk[2 * z + 1] = (int)pf + 1;
        gq[z] = vi - pf;
      }
    }
    // target bucket of each order statistic: last b with start[b] <= k (broadcast reads)
    int tb[4], ts0[4], tn[4];
    bool slow = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int l = 0, h = NB + 1;
      while (l < h) {
        const int m = (l + h) >> 1;
        if ((int)fr_cnt_get(cnt, m) <= kk[j]) l = m + 1; else h = m;
      }
      tb[j] = l - 1;
      ts0[j] = (int)fr_cnt_get(cnt, tb[j]);
      tn[j] = (int)fr_cnt_get(cnt, tb[j] + 1) - ts0[j];
      slow |= (tb[j] % (K + 1)) != K && tn[j] > FR_QCAP;
    }
    __syncthreads();                          // counters dead: the lists reuse their LDS
    if (!slow) {
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (bb[k] == tb[j] && (tb[j] % (K + 1)) != K) lists[j * FR_QCAP + atomicAdd(&tfill[j], 1)] = key[k];
      }
      __syncthreads();
      if (wid < 4) {
        const int j = wid, b = tb[j];
        if ((b % (K + 1)) == K) {
          if (lane == 0) tval[j] = tab.spl[b / (K + 1)];
        } else {
          const uint64_t* L = lists + j * FR_QCAP;
          const int n = tn[j], r = kk[j] - ts0[j];
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
    if (!fr_in<NT>(t, k, (int)A)) continue;
    const double v = key[k] == KEY_SENTINEL ? qnan() : okey_inv(key[k]);
    double o;
    if (OP == 0) {
      o = v;
      if (nv >= 5) o = (v < lo) ? lo : ((v > hi) ? hi : v);
    } else {
      o = (v < lo || v > hi) ? v : 0.0;
    }
    y[t + k * NT] = (PRES && !((pm >> k) & 1)) ? qnan() : o;
  }
}

// Thread 0 of an IC workgroup: the (n, IC, rank IC, beta) records of source row s for its
// active lags from the block totals (cst: -min / max of f and r per lag, fin: the seven
// moment sums per lag).
__device__ __forceinline__ void fr_ic_store(double* out, int64_t F, int64_t D, int64_t s, int64_t f,
                                            const int* lagv, const bool* act, const double* n,
                                            const double* cst, const double* fin) {
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    if (!act[m]) continue;
    const int64_t td = s + lagv[m];
    double* o = out + ((int64_t)(m * 4) * F + f) * D + td;
    const int64_t stp = F * D;
    const double nn = n[m];
    double ic = qnan(), ric = qnan(), beta = qnan();
    if (nn >= 3.0) {
      const double* w = fin + 8 * m;
      const bool fconst = (-cst[4 * m + 0]) == cst[4 * m + 1];
      const bool rconst = (-cst[4 * m + 2]) == cst[4 * m + 3];
      if (!fconst && !rconst) {
        ic = fmin(1.0, fmax(-1.0, w[0] / sqrt(w[1] * w[2])));
        ric = fmin(1.0, fmax(-1.0, w[3] / sqrt(w[4] * w[2])));
      }
      beta = w[5] > 0 ? w[6] / w[5] : qnan();
    }
    o[0] = nn;
    o[stp] = ic;
    o[2 * stp] = ric;
    o[3 * stp] = beta;
  }
}

// ------------------------------------------------------------------------------------
// Fused daily IC: workgroup (source row s, factor f) ranks X[f][s] once and produces the
// stats of the pairs (X[f][s], R[s + L_m]) for up to two lags.  Bucket members are the
// exposures pair-valid for at least one lag; one 64-bit counter per bucket packs
// (#members | #lag-0 members << 16 | #lag-1 members << 32), so a single atomic gives the
// scatter slot and a single scan gives both lags' rank bases.
// Output: out[((m*4 + j) * F + f) * D + s + L_m], j = n, IC, rank IC, beta.
// Occupancy target: two 1024-thread rows per CU (64 VGPRs) while the row's LDS allows it
// (A <= 5120); longer rows hold one row per CU anyway (LDS), so they get 128 VGPRs.
template <int NT, int EMAX>
__global__ void __launch_bounds__(NT, (NT == 1024 && EMAX <= 5) ? 8 : 4)
k_ic_daily_fr(const double* __restrict__ X, const double* __restrict__ Rt, int64_t F, int64_t D, int64_t A,
              int64_t ld, int L0, int L1, int NL, double* __restrict__ out) {
  constexpr int K = FR_K_IC, NB = FRG<K>::NB, NW = NT / 64;
  // packed per-element state: slot (14 bits) | bucket << 14 (13 bits) | lag mask << 27
  constexpr int FR_MSH = 27, FR_BMASK = 0x1fff;
  static_assert(NB <= FR_BMASK, "bucket id field");
  using u64 = unsigned long long;
  __shared__ FrTab tab;
  __shared__ u64 uscr[NW];
  __shared__ double dscr[(NW + 1) * 16];
  // one dynamic buffer, two lives: the NB+1 packed bucket counters, then (once every
  // element has read its counters) the bucket-ordered keys [A], member info [A] and lag
  // masks [A] of the in-bucket scan
  extern __shared__ uint64_t lds[];
  u64* cnt = (u64*)lds;
  uint64_t* bkey = lds;
  uint32_t* binfo = (uint32_t*)(bkey + A);    // bucket start | member count << 16 (0: no scan)
  uint8_t* bmask = (uint8_t*)(binfo + A);
  const int t = threadIdx.x, wid = t >> 6;
  BR_PH_INIT;
  // date-major rows: the F workgroups of a date share its return rows in L2 (measured
  // faster than factor-major order at C2: 44.8 vs 46.5 ms)
  const int64_t s = fmx_blk() / F, f = fmx_blk() % F;   // grid dim3(F, D)
  const double* xf = X + (f * D + s) * ld;
  const int lagv[2] = {L0, L1};
  const double* rr[2];
  bool act[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    act[m] = m < NL && s + lagv[m] < D;
    rr[m] = Rt + (act[m] ? s + lagv[m] : s) * ld;   // always a valid row
  }
  if (!act[0] && !act[1]) return;
  uint64_t key[EMAX];
  int pk[EMAX];                               // mask << FR_MSH, later slot | bucket
  // v1: sum f, sum r of lag 0, then of lag 1 (pair counts come from ballots);
  // mx: -min f, max f, -min r, max r per lag
  double v1[4] = {0, 0, 0, 0};
  double mx[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) mx[q] = -INFINITY;
  int cw0 = 0, cw1 = 0;                       // wave-uniform pair counts per lag
  // the row's exposures are all in flight before the first is consumed
  double xv[EMAX];
#pragma unroll
  for (int k = 0; k < EMAX; ++k) xv[k] = fr_in<NT>(t, k, (int)A) ? xf[t + k * NT] : qnan();
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int i = t + k * NT;
    key[k] = KEY_SENTINEL;
    pk[k] = 0;
    int mm = 0;
    const double v = xv[k];
    if (v == v) {
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        if (!act[m]) continue;
        const double r = rr[m][i];
        if (r != r) continue;
        mm |= 1 << m;
        v1[2 * m] += v;
        v1[2 * m + 1] += r;
        mx[4 * m + 0] = fmax(mx[4 * m + 0], -v);
        mx[4 * m + 1] = fmax(mx[4 * m + 1], v);
        mx[4 * m + 2] = fmax(mx[4 * m + 2], -r);
        mx[4 * m + 3] = fmax(mx[4 * m + 3], r);
      }
      if (mm) { key[k] = okey(v); pk[k] = mm << FR_MSH; }
    }
    cw0 += __popcll(__ballot(mm & 1));
    cw1 += __popcll(__ballot(mm & 2));
  }
  const uint64_t smp = wid == 0 ? fr_sample(xf, nullptr, A) : KEY_SENTINEL;
  for (int b = t; b <= NB; b += NT) cnt[b] = 0;
  fr_part_bfly<4, false>(v1, dscr, 16, 0);
  if ((t & 63) == 0) {
    dscr[wid * 16 + 4] = (double)cw0;
    dscr[wid * 16 + 5] = (double)cw1;
    dscr[wid * 16 + 6] = 0.0;
    dscr[wid * 16 + 7] = 0.0;
  }
  fr_part_bfly<8, true>(mx, dscr, 16, 8);
  fr_fin_dpp<NT>(dscr, 16, 8);
  const double* tot1 = dscr + NW * 16;        // f0, r0, f1, r1 sums, n0, n1 [0,6); -min/max [8,16)
  double tot[6];                              // block-uniform: kept in SGPRs
#pragma unroll
  for (int q = 0; q < 6; ++q) tot[q] = fr_uniform_d(tot1[q]);
  BR_PH();
  __shared__ double cst[8];                   // only thread 0 reads them back
  if (t == 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) cst[q] = tot1[8 + q];
  }
  // pair counts as (exact) doubles: they stay in SGPRs, an int copy would live in VGPRs
  const double n[2] = {tot[4], tot[5]};
  const bool need = (act[0] && n[0] >= 3.0) || (act[1] && n[1] >= 3.0);
  __shared__ double fin[16];                  // per-lag moment totals (thread 0)
  if (need) {
    if (wid == 0) {
      // bounds of the union of both lags' members (empty lag: -min = max = -inf)
      const double vmin = -fmax(tot1[8], tot1[12]), vmax = fmax(tot1[9], tot1[13]);
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
    // Counters -> registers: a0[k] / a1[k] = the lag's rank base (members of lower
    // buckets) | #equal << 16 for elements whose bucket needs no scan.  pk[k] becomes the
    // element's slot in bucket order (every pair-valid element has a unique one) | lag
    // mask << FR_MSH.  Elements of buckets to scan park the member count in a0's #equal
    // half and the bucket start in a1 bits 14..27, flagged by a1's sign bit.
    int a0[EMAX], a1[EMAX];
    const int nmem = (int)(cnt[NB] & 0xffff);   // pair-valid elements (either lag)
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      a0[k] = 0; a1[k] = 0;
      if (key[k] == KEY_SENTINEL) continue;
      const int b = (pk[k] >> PK_BSHIFT) & FR_BMASK;
      const int mk = pk[k] >> FR_MSH;
      const u64 c0 = cnt[b], dc = cnt[b + 1] - c0;
      const int nall = (int)(dc & 0xffff);
      const int s0 = (int)(c0 & 0xffff);
      const int b0 = (int)((c0 >> 16) & 0xffff), b1 = (int)((c0 >> 32) & 0xffff);
      if ((b % (K + 1)) == K) {
        a0[k] = b0 | ((int)((dc >> 16) & 0xffff) << 16);
        a1[k] = b1 | ((int)((dc >> 32) & 0xffff) << 16);
      } else if (nall == 1) {
        a0[k] = b0 | ((mk & 1) << 16);
        a1[k] = b1 | ((mk >> 1) << 16);
      } else {
        a0[k] = b0 | (nall << 16);
        a1[k] = b1 | (s0 << 14) | (int)0x80000000u;
      }
      pk[k] = (s0 + (pk[k] & PK_SLOT)) | (mk << FR_MSH);
    }
    __syncthreads();                          // counters dead: bucket-ordered arrays reuse them
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (key[k] == KEY_SENTINEL) continue;
      const int q = pk[k] & PK_SLOT;
      const bool scan = a1[k] < 0;
      bkey[q] = key[k];
      binfo[q] = scan ? ((uint32_t)((a1[k] >> 14) & 0x3fff) | ((uint32_t)a0[k] & 0xffff0000u)) : 0u;
      bmask[q] = (uint8_t)(pk[k] >> FR_MSH);
      if (scan) { a0[k] &= 0xffff; a1[k] &= 0x3fff; }
    }
    __syncthreads();
    BR_PH();
    // In-bucket scan, position-parallel: thread t takes bucket-ordered slots t + i*NT, so a
    // large bucket (tie cluster, dense tail) is spread over consecutive lanes of one or two
    // waves instead of stretching every wave's loop.  res = #less | #equal << 16 per lag;
    // lag 0's goes straight into the slot's own binfo word (read only by its owner), lag
    // 1's over the key after a barrier.  Slots of buckets without a scan end with 0 in both.
    uint32_t res1[EMAX];
#pragma unroll
    for (int i = 0; i < EMAX; ++i) {
      res1[i] = 0;
      const int q = t + i * NT;
      if (q >= nmem) continue;
      const uint32_t in = binfo[q];
      const int len = (int)(in >> 16);
      if (len == 0) continue;
      const int st = (int)(in & 0xffff);
      const uint64_t me = bkey[q];
      uint32_t r0 = 0;
      for (int j = 0; j < len; ++j) {
        const uint64_t w = bkey[st + j];
        const uint32_t wm = bmask[st + j];
        const uint32_t inc = (w < me ? 1u : 0u) + (w == me ? 0x10000u : 0u);
        r0 += (wm & 1) ? inc : 0u;
        res1[i] += (wm & 2) ? inc : 0u;
      }
      binfo[q] = r0;
    }
    __syncthreads();                          // all scans done: lag-1 results overwrite the keys
    uint32_t* bres1 = reinterpret_cast<uint32_t*>(bkey);
#pragma unroll
    for (int i = 0; i < EMAX; ++i) {
      const int q = t + i * NT;
      if (q < nmem) bres1[2 * q] = res1[i];
    }
    __syncthreads();
    BR_PH();
    // pk[k] <- 2*rank(lag 0) | 2*rank(lag 1) << 16 (half-integer ranks, exact); a field is
    // 0 when the element is not a member of that lag's pairs
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (key[k] == KEY_SENTINEL) continue;
      const int mk = pk[k] >> FR_MSH;
      a0[k] += (int)binfo[pk[k] & PK_SLOT];
      a1[k] += (int)bres1[2 * (pk[k] & PK_SLOT)];
      pk[k] = ((mk & 1) ? (2 * (a0[k] & 0xffff) + (a0[k] >> 16) + 1) : 0) |
              ((mk & 2) ? ((2 * (a1[k] & 0xffff) + (a1[k] >> 16) + 1) << 16) : 0);
    }
    double fm[2], rm[2], km[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const double dn = n[m];
      fm[m] = tot[2 * m] / dn;
      rm[m] = tot[2 * m + 1] / dn;
      km[m] = (dn + 1.0) / 2.0;
    }
    BR_PH();
    // one lag at a time keeps 7 accumulators live
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      double w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
        const int r2 = key[k] == KEY_SENTINEL ? 0 : (m == 0 ? (pk[k] & 0xffff) : (int)((unsigned)pk[k] >> 16));
        if (r2 == 0) continue;
        const int64_t i = t + (int64_t)k * NT;
        const double fv = okey_inv(key[k]);
        const double rk = (double)r2 / 2.0;
        const double r = rr[m][i];
        const double dx = fv - fm[m], dy = r - rm[m], dk = rk - km[m];
        w[0] += dx * dy; w[1] += dx * dx; w[2] += dy * dy;
        w[3] += dk * dy; w[4] += dk * dk;
        w[5] += fv * fv; w[6] += fv * r;
      }
      fr_part_bfly<8, false>(w, dscr, 16, 8 * m);
    }
    fr_fin_dpp<NT>(dscr, 16, 16);
    if (t < 16) fin[t] = dscr[NW * 16 + t];
    __syncthreads();
  }
  if (t == 0) fr_ic_store(out, F, D, s, f, lagv, act, n, cst, fin);
  BR_PH();
}

// ------------------------------------------------------------------------------------
// Daily IC from the ranks the cs_rank pass of the same panel already produced (RK =
// 2*#less + #equal + 1 among the row's non-NaN exposures, k_cs_rank_fa), so no sort or
// histogram is repeated.  The pairs of lag m are the non-NaN exposures minus E_m, those
// whose lag-m return is NaN; the doubled pair rank is RK - (2*#less + #equal) over E_m
// (#less + #less-or-equal: exactly the correction).
//
// ic_ranked_row: one 1024-thread workgroup per row, any E_m -- the rows the wave kernel
// (k_ic_wave, below) hands over.  E_m keys gathered in LDS while the row loads, sorted by
// one wave when < 64 (a sentinel ends the list) and binary-searched; a longer E_m is
// counting-sorted by 64-rank blocks of the members' doubled ranks (O(A + |E|)).  Sums and two-pass moments as in
// k_ic_daily_fr (same element order, same butterflies: the records are bit-identical).
template <int NT, int EMAX>
__device__ __forceinline__ void ic_ranked_row(int64_t row, const double* __restrict__ X,
                                              const fmx_rank2_t* __restrict__ RK, const double* __restrict__ Rt,
                                              int64_t F, int64_t D, int64_t A, int64_t ld, int L0, int L1, int NL,
                                              double* __restrict__ out) {
  constexpr int NW = NT / 64, ES = 64;
  __shared__ double dscr[(NW + 1) * 16];
  __shared__ uint64_t el[2][ES];              // E_m keys (first ES), then sorted
  __shared__ uint32_t ltbl[(2 * 16384 >> 6) + 2];   // long E_m: 64-rank block table (A <= 16384)
  __shared__ uint32_t lent[16384];                 //            entries grouped by block
  __shared__ int ecnt[2], wcnt[NW];
  __shared__ double cst[8], fin[16];
  const int t = threadIdx.x, wid = t >> 6, lane = t & 63;
  BR_PH_INIT;
  const int64_t s = row / F, f = row % F;
  const double* xf = X + (f * D + s) * ld;
  const fmx_rank2_t* rkf = RK + (f * D + s) * ld;
  const int lagv[2] = {L0, L1};
  const double* rr[2];
  bool act[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    act[m] = m < NL && s + lagv[m] < D;
    rr[m] = Rt + (act[m] ? s + lagv[m] : s) * ld;
  }
  if (!act[0] && !act[1]) return;
  if (t < 2) ecnt[t] = 0;
  double v1[4] = {0, 0, 0, 0};
  double mx[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) mx[q] = -INFINITY;
  int cw0 = 0, cw1 = 0;
  double xv[EMAX];
#pragma unroll
  for (int k = 0; k < EMAX; ++k) xv[k] = fr_in<NT>(t, k, (int)A) ? xf[t + k * NT] : qnan();
  __syncthreads();                            // ecnt zeroed
  uint32_t pm = 0, em = 0;                    // per element: pair / E mask of each lag
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int i = t + k * NT;
    int mm = 0, ee = 0;
    const double v = xv[k];
    if (v == v) {
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        if (!act[m]) continue;
        const double r = rr[m][i];
        if (r != r) { ee |= 1 << m; continue; }
        mm |= 1 << m;
        v1[2 * m] += v;
        v1[2 * m + 1] += r;
        mx[4 * m + 0] = fmax(mx[4 * m + 0], -v);
        mx[4 * m + 1] = fmax(mx[4 * m + 1], v);
        mx[4 * m + 2] = fmax(mx[4 * m + 2], -r);
        mx[4 * m + 3] = fmax(mx[4 * m + 3], r);
      }
      if (ee) {                               // rare: the row's NaN returns
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          if (!((ee >> m) & 1)) continue;
          const int q = atomicAdd(&ecnt[m], 1);
          if (q < ES) el[m][q] = okey(v);
        }
      }
    }
    pm |= (uint32_t)mm << (2 * k);
    em |= (uint32_t)ee << (2 * k);
    cw0 += __popcll(__ballot(mm & 1));
    cw1 += __popcll(__ballot(mm & 2));
  }
  BR_PH();
  fr_part_bfly<4, false>(v1, dscr, 16, 0);
  if ((t & 63) == 0) {
    dscr[wid * 16 + 4] = (double)cw0;
    dscr[wid * 16 + 5] = (double)cw1;
    dscr[wid * 16 + 6] = 0.0;
    dscr[wid * 16 + 7] = 0.0;
  }
  fr_part_bfly<8, true>(mx, dscr, 16, 8);
  fr_fin_dpp<NT>(dscr, 16, 8);
  const double* tot1 = dscr + NW * 16;
  double tot[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) tot[q] = fr_uniform_d(tot1[q]);
  if (t == 0) {
#pragma unroll
    for (int q = 0; q < 8; ++q) cst[q] = tot1[8 + q];
  }
  const double n[2] = {tot[4], tot[5]};
  const bool need = (act[0] && n[0] >= 3.0) || (act[1] && n[1] >= 3.0);
  BR_PH();
  if (need) {
    // doubled ranks (loads in flight over the E sort)
    uint32_t rk[EMAX];
#pragma unroll
    for (int k = 0; k < EMAX; ++k) rk[k] = fr_in<NT>(t, k, (int)A) ? rkf[t + k * NT] : 0u;
    const int ne[2] = {__builtin_amdgcn_readfirstlane(ecnt[0]), __builtin_amdgcn_readfirstlane(ecnt[1])};
    const int nw = wid == 0 ? ne[0] : ne[1];
    if (wid < 2 && nw > 0 && nw < ES) {
      const uint64_t v = lane < nw ? el[wid][lane] : KEY_SENTINEL;
      el[wid][lane] = wave_sort64(v, lane);
    }
    __syncthreads();
    BR_PH();
    // cr[k] = doubled pair rank of lag 0 | lag 1 << 16: RK minus the E corrections (every
    // partial difference stays >= the final one >= 2, so the fields never borrow)
    uint32_t cr[EMAX];
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      cr[k] = rk[k] | (rk[k] << 16);
      if (!((pm >> (2 * k)) & 3)) continue;
      const uint64_t key = okey(xv[k]);
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        if (!((pm >> (2 * k + m)) & 1) || ne[m] == 0 || ne[m] >= ES) continue;
        int lo = 0, le = 0;
#pragma unroll
        for (int st = ES / 2; st > 0; st >>= 1) {
          lo += el[m][lo + st - 1] < key ? st : 0;
          le += el[m][le + st - 1] <= key ? st : 0;
        }
        cr[k] -= (uint32_t)(lo + le) << (16 * m);
      }
    }
    // long E_m (any size): counting-sort the E members' doubled ranks into 64-rank blocks
    // (key order = rank order within the row) -- the same table as k_ic_wave, so each pair
    // element's correction is 2 * #entries of earlier blocks + a scan of its own block's
    // (few) entries: O(A + |E|) per row instead of O(A * |E|)
    const int nb = (int)((2 * A) >> 6) + 1;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      if (ne[m] < ES) continue;               // block-uniform
      for (int b = t; b < nb; b += NT) ltbl[b] = 0u;
      __syncthreads();
      int sl[EMAX];
#pragma unroll
      for (int k = 0; k < EMAX; ++k)
        sl[k] = ((em >> (2 * k + m)) & 1) ? (int)atomicAdd(&ltbl[rk[k] >> 6], 1u) : 0;
      __syncthreads();
      {
        // exclusive scan of the block counts, NT >= nb (A <= 16384 -> nb <= 513)
        const int n = t < nb ? (int)ltbl[t] : 0;
        int tot;
        const int st0 = block_exscan<NT>(n, wcnt, &tot);
        if (t < nb) ltbl[t] = (uint32_t)st0 | ((uint32_t)(st0 + n) << 16);
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < EMAX; ++k)
        if ((em >> (2 * k + m)) & 1) lent[(ltbl[rk[k] >> 6] & 0xffffu) + sl[k]] = rk[k];
      __syncthreads();
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
        if (!((pm >> (2 * k + m)) & 1)) continue;
        const uint32_t tb2 = ltbl[rk[k] >> 6];
        const uint32_t j0 = tb2 & 0xffffu, j1 = tb2 >> 16;
        uint32_t a = 2u * j0;
        for (uint32_t j = j0; j < j1; ++j) {
          const uint32_t e = lent[j];
          a += (e < rk[k] ? 1u : 0u) + (e <= rk[k] ? 1u : 0u);
        }
        cr[k] -= a << (16 * m);
      }
      __syncthreads();                        // the table is reused by the next lag
    }
    BR_PH();
    double fm[2], rm[2], km[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const double dn = n[m];
      fm[m] = tot[2 * m] / dn;
      rm[m] = tot[2 * m + 1] / dn;
      km[m] = (dn + 1.0) / 2.0;
    }
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      double w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < EMAX; ++k) {
        if (!((pm >> (2 * k + m)) & 1)) continue;
        const int r2 = (int)((cr[k] >> (16 * m)) & 0xffff);
        const int64_t i = t + (int64_t)k * NT;
        const double fv = xv[k];
        const double rkv = (double)r2 / 2.0;
        const double r = rr[m][i];
        const double dx = fv - fm[m], dy = r - rm[m], dk = rkv - km[m];
        w[0] += dx * dy; w[1] += dx * dx; w[2] += dy * dy;
        w[3] += dk * dy; w[4] += dk * dk;
        w[5] += fv * fv; w[6] += fv * r;
      }
      fr_part_bfly<8, false>(w, dscr, 16, 8 * m);
    }
    BR_PH();
    fr_fin_dpp<NT>(dscr, 16, 16);
    if (t < 16) fin[t] = dscr[NW * 16 + t];
    __syncthreads();
  }
  if (t == 0) fr_ic_store(out, F, D, s, f, lagv, act, n, cst, fin);
  BR_PH();
}

// The rows listed by k_ic_wave (list[0] = count, then row ids): a grid of workgroups
// walks the list.
template <int NT, int EMAX>
__global__ void __launch_bounds__(NT, 4)
k_ic_ranked_list(const double* __restrict__ X, const fmx_rank2_t* __restrict__ RK, const double* __restrict__ Rt,
                 int64_t F, int64_t D, int64_t A, int64_t ld, int L0, int L1, int NL, double* __restrict__ out,
                 const int32_t* __restrict__ list) {
  const int n = list[0];
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    ic_ranked_row<NT, EMAX>(list[1 + i], X, RK, Rt, F, D, A, ld, L0, L1, NL, out);
    __syncthreads();                          // LDS reused by the next row
  }
}

}  // namespace fmx
