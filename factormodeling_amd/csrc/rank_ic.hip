// Fused two-lag daily IC launcher (rank_kernels.hpp).
// Reference: factor_selector.py:36-48
#include "rank_fine.hpp"
#include "rank_launch.hpp"

namespace fmx {

// dates t < L get an empty record (n = 0, NaN stats)
__global__ void k_ic_empty(double* out, int64_t F, int64_t D, int L0, int L1, int NL) {
  const int64_t f = blockIdx.x;
  for (int m = 0; m < NL; ++m) {
    const int L = m == 0 ? L0 : L1;
    for (int64_t td = threadIdx.x; td < min<int64_t>(L, D); td += blockDim.x) {
      double* o = out + ((int64_t)(m * 4) * F + f) * D + td;
      o[0] = 0.0;
      o[F * D] = qnan();
      o[2 * F * D] = qnan();
      o[3 * F * D] = qnan();
    }
  }
}


fmx_status br_ic_daily(const double* X, const double* R, int64_t F, int64_t D, int64_t A, int64_t ld,
                       const int32_t* lags_host, int n_lags, double* out, hipStream_t st) {
  // 512-thread rows up to 4096 assets (C4's 3000: 20.0 vs 23.7 ms per 252 dates)
  const int nt = br_nt(A <= 4096 ? 512 : 1024);
  // counters, then keys [A] + member info [A] + lag masks [A] (k_ic_daily_fr)
  const size_t lds_fr = std::max<size_t>((size_t)(FRG<FR_K_IC>::NB + 1) * 8, (size_t)A * 13 + 16);
  auto fr_table = FMX_EMAX_TABLE(k_ic_daily_fr);
  const bool fine = rank_impl() == RANK_IMPL_FINE && lds_fits(fr_table(nt, br_emax(A, nt)), lds_fr);
  const size_t lds = fine ? lds_fr : (size_t)std::max<int64_t>(A, nt) * 8 + (size_t)((A + 15) & ~15ll);
  if (!fine && !lds_fits(FMX_EMAX_TABLE(k_ic_daily_br)(nt, br_emax(A, nt)), lds)) {
    set_error("row too long for the IC kernels' LDS (rank it once with fmx_cs_rank_winsor and use "
              "fmx_ic_daily_ranked)");
    return FMX_ERR_UNSUPPORTED;
  }
  for (int base = 0; base < n_lags; base += 2) {
    int NL = std::min(2, n_lags - base);
    int L0 = lags_host[base], L1 = NL > 1 ? lags_host[base + 1] : 0;
    double* o = out + (int64_t)base * 4 * F * D;
    k_ic_empty<<<(unsigned)F, 64, 0, st>>>(o, F, D, L0, L1, NL);
    FMX_LAUNCH_CHECK("k_ic_empty");
    void* args[] = {(void*)&X, (void*)&R, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&L0, (void*)&L1,
                    (void*)&NL, (void*)&o};
    // date-major rows (s = row / F): grid dim3(F, D)
    fmx_status e = fine ? launch_br(fr_table, nt, A, F, D, lds, args, st)
                        : launch_br(FMX_EMAX_TABLE(k_ic_daily_br), nt, A, F, D, lds, args, st);
    if (e) return e;
  }
  return FMX_OK;
}

// ------------------------------------------------------------------------------------
// NaN-return positions per date (the candidates of every row's E lists): one wave per
// date, ballot-compacted in asset order; npos[t] = the full count, pos[t][0..ICW_PC) the
// first ICW_PC positions.
constexpr int ICW_PC = 256;
__global__ void __launch_bounds__(256)
k_nan_positions(const double* __restrict__ Rt, int64_t D, int64_t A, int64_t ld, int32_t* __restrict__ pos,
                int32_t* __restrict__ npos) {
  const int lane = threadIdx.x & 63;
  const int64_t d = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (d >= D) return;
  const double* r = Rt + d * ld;
  const uint64_t lt = (1ull << lane) - 1ull;
  int c = 0;
  for (int64_t i0 = 0; i0 < A; i0 += 64) {
    const int64_t i = i0 + lane;
    const bool nan = i < A && !(r[i] == r[i]);
    const uint64_t b = __ballot(nan);
    const int at = c + __popcll(b & lt);
    if (nan && at < ICW_PC) pos[d * ICW_PC + at] = (int32_t)i;
    c += __popcll(b);
  }
  if (lane == 0) npos[d] = c;
}

// ------------------------------------------------------------------------------------
// Daily IC from the ranks, one WAVE per row: no workgroup barrier anywhere, so ~20 rows
// are in flight per CU instead of two 1024-thread rows.
//  1. E_m from the target date's NaN-return positions (<= ICW_PC of them, else the row
//     goes to the overflow list for ic_ranked_row): the doubled ranks of the valid
//     exposures there, counting-sorted into 64-rank blocks in LDS.
//  2. one streaming pass over x, RK and the two return rows: per lag, the pair count
//     (ballots) and sums shifted by the lag's first pair (single-pass moments without
//     cancellation; constant inputs = nothing differs from that pair); the pair rank is
//     RK minus the E correction read off the rank-block table.
//  3. multi-value DPP butterflies, lane 0 writes the records.
// Moments are single-pass about the first pair (rank moments from exact integer sums), so
// records agree with the two-pass kernels to ~1e-15 relative, not bitwise.
constexpr int ICW_WAVES = 4;
#ifndef ICW_PF
#define ICW_PF 1
#endif
constexpr int ICW_EC = 256;   // E entries per (wave, lag); more NaN returns: ICW_PC overflow
// table word of a block without a first / second entry: both entry fields 0xffff (no doubled
// rank reaches it: ranks <= 2A <= 32768), so the per-element correction needs no count tests
constexpr uint64_t ICW_NO_ENTRY = 0xffffffff00000000ull;

#ifndef ICW_MINW
#define ICW_MINW 6
#endif
__global__ void __launch_bounds__(64 * ICW_WAVES, ICW_MINW)
k_ic_wave(const double* __restrict__ X, const fmx_rank2_t* __restrict__ RK, const double* __restrict__ Rt, int64_t F,
          int64_t D, int64_t A, int64_t ld, int L0, int L1, int NL, double* __restrict__ out,
          const int32_t* __restrict__ pos, const int32_t* __restrict__ npos, int32_t* __restrict__ ovf) {
  // per wave and lag: the rank-block table T[nbp] (block b = doubled ranks [64b, 64b+64))
  // and the entries eb[ICW_EC] grouped by block.  T[b] is 64-bit: 2 * start | count << 16
  // of its E entries in eb (2 * start = the correction of every earlier block's entries), and
  // the block's first two entries (<< 32, << 48; entries are doubled ranks in [2, 2A], 16
  // bits; 0xffff where absent): one ds_read_b64 per lag and element instead of the table
  // word plus two entry reads.  Dynamic LDS: ICW_WAVES * 2 * (2 nbp + ICW_EC) + 2 words.
  extern __shared__ uint32_t icw_lds[];
  __shared__ double scr[ICW_WAVES * 32];
  // the wave index as a scalar: the row, its pointers and lags live in SGPRs (saddr loads)
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t row = (int64_t)blockIdx.x * ICW_WAVES + wid;
  if (row >= F * D) return;                   // whole waves; no workgroup barrier below
  const int64_t s = row / F, f = row % F;
  const int lagv[2] = {L0, L1};
  const double* rr[2];
  bool act[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    act[m] = m < NL && s + lagv[m] < D;
    rr[m] = Rt + (act[m] ? s + lagv[m] : s) * ld;
  }
  if (!act[0] && !act[1]) return;
  const double* xf = X + (f * D + s) * ld;
  const fmx_rank2_t* rkf = RK + (f * D + s) * ld;
  const int nb = (int)((2 * A) >> 6) + 1;     // doubled ranks are <= 2A
  const int nbp = (nb + 1) & ~1;
  uint32_t* T[2];                             // counts during the build (u32 view of T64)
  uint64_t* T64[2];
  uint32_t* eb[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    T[m] = icw_lds + (wid * 2 + m) * (2 * nbp + ICW_EC);
    T64[m] = reinterpret_cast<uint64_t*>(T[m]);
    eb[m] = T[m] + 2 * nbp;
  }
  // 1. E lists: the doubled ranks of the valid exposures at the target date's NaN-return
  // positions (key(e) < key(x) <=> RK(e) < RK(x), ties alike, so the corrections can be
  // counted on ranks), counting-sorted by rank block: per element the correction is then
  // 2 * (#entries of earlier blocks) + one (usually empty) scan of its own block's entries,
  // one LDS read instead of a binary search (the searches were LDS-bound: 2 lags x 7 reads).
  int ne[2] = {0, 0};
  bool over = false;
  uint32_t er[2][ICW_EC / 64];                // this lane's entries (0: none) and their slots
  int es[2][ICW_EC / 64];
  // the first chunk of the streaming pass (step 2) is in flight during the E-list setup
  const int An = (int)A;
  double xq[ICW_PF], rq[ICW_PF][2];
  uint32_t kq[ICW_PF];
  // an inactive lag reads the row's own date (rr clamped above): its sums are never written
  auto load = [&](int i0, int s) {
    const int i = i0 + lane;
    if (i0 + 64 <= An) {                      // wave-uniform: every chunk but a ragged last
      xq[s] = xf[i];
      kq[s] = (uint32_t)rkf[i];
#pragma unroll
      for (int m = 0; m < 2; ++m) rq[s][m] = rr[m][i];
    } else {
      const bool in = i < An;
      xq[s] = in ? xf[i] : qnan();
      kq[s] = in ? (uint32_t)rkf[i] : 0u;
#pragma unroll
      for (int m = 0; m < 2; ++m) rq[s][m] = in ? rr[m][i] : qnan();
    }
  };
#pragma unroll
  for (int s = 0; s < ICW_PF; ++s) load(64 * s, s);
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    for (int b = lane; b < nbp; b += 64) T64[m][b] = 0ull;
#pragma unroll
    for (int q = 0; q < ICW_EC / 64; ++q) { er[m][q] = 0u; es[m][q] = 0; }
  }
  __builtin_amdgcn_wave_barrier();
  // both lags' lists at once: their (independent) position and rank loads overlap
  int cl[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) cl[m] = act[m] ? npos[s + lagv[m]] : 0;
  over = cl[0] > ICW_PC || cl[1] > ICW_PC;
  if (!over) {
    const int cmax = cl[0] > cl[1] ? cl[0] : cl[1];
    const int32_t* pp[2] = {pos + (s + (act[0] ? lagv[0] : 0)) * ICW_PC, pos + (s + (act[1] ? lagv[1] : 0)) * ICW_PC};
#pragma unroll
    for (int q = 0; q < ICW_EC / 64; ++q) {
      if (64 * q >= cmax) break;              // wave-uniform
      const int j = 64 * q + lane;
      int p[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) p[m] = pp[m][j];                 // unconditional (j < ICW_PC)
#pragma unroll
      for (int m = 0; m < 2; ++m) p[m] = j < cl[m] ? p[m] : 0;      // valid positions only
      uint32_t r2[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) r2[m] = (uint32_t)rkf[p[m]];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const uint32_t e = j < cl[m] ? r2[m] : 0u;                  // 0: NaN exposure / no entry
        er[m][q] = e;
        if (e) es[m][q] = (int)atomicAdd(&T[m][e >> 6], 1u);
        ne[m] += __popcll(__ballot(e != 0u));
      }
    }
  }
  if (over) {                                 // > ICW_PC NaN returns: the workgroup kernel takes the row
    if (lane == 0) {
      const int q = atomicAdd(&ovf[0], 1);
      ovf[1 + q] = (int32_t)row;
    }
    return;
  }
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    if (ne[m] == 0) continue;                 // wave-uniform
    // exclusive scan of the block counts: lane l owns blocks [l R, l R + R) (R <= 9: A <= 16384)
    constexpr int RMAX = 9;
    const int R = (nbp + 63) >> 6;
    int cn[RMAX];
    int loc = 0;
#pragma unroll
    for (int q = 0; q < RMAX; ++q) {
      const int b = lane * R + q;
      cn[q] = (q < R && b < nbp) ? (int)T[m][b] : 0;   // the u32 counts, read before T64 is written
      loc += cn[q];
    }
    int incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = fr_up(incl, o, lane);
      if (lane >= o) incl += u;
    }
    int run = incl - loc;
    int st[RMAX];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < RMAX; ++q) {
      const int b = lane * R + q;
      st[q] = run;
      if (q < R && b < nbp) T64[m][b] = ICW_NO_ENTRY | (uint64_t)((uint32_t)(2 * run) | ((uint32_t)cn[q] << 16));
      run += cn[q];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < ICW_EC / 64; ++q)
      if (er[m][q]) eb[m][(((uint32_t)T64[m][er[m][q] >> 6] & 0xffffu) >> 1) + es[m][q]] = er[m][q];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // the first two entries of each block into its table word
#pragma unroll
    for (int q = 0; q < RMAX; ++q) {
      const int b = lane * R + q;
      if (q < R && b < nbp && cn[q] > 0) {
        const uint64_t e0 = eb[m][st[q]], e1 = cn[q] > 1 ? eb[m][st[q] + 1] : 0xffffu;
        T64[m][b] = (uint64_t)((uint32_t)(2 * st[q]) | ((uint32_t)cn[q] << 16)) | (e0 << 32) | (e1 << 48);
      }
    }
  }
#pragma unroll
  for (int m = 0; m < 2; ++m)                 // a lag without entries: every block empty
    if (ne[m] == 0)
      for (int b = lane; b < nbp; b += 64) T64[m][b] = ICW_NO_ENTRY;
  __builtin_amdgcn_wave_barrier();
  // 2. one pass.  Per lag: pair count (ballots); the first pair's (x, r) is the lag's
  // shift (a, b) and reference (constant inputs: no pair differs from it); sums of x', r',
  // x'^2, r'^2, x'r' (x' = x - a, r' = r - b), of 2k * r' and (2k)^2 (exact integers) with
  // 2k = RK minus the E correction.
  double sm[2][6];
  uint64_t kk[2] = {0, 0};
  double ax[2] = {0.0, 0.0}, ar[2] = {0.0, 0.0};
  bool ref[2] = {false, false};
  int cnt[2] = {0, 0};
  uint64_t dm[4] = {0, 0, 0, 0};              // [2m]: lanes whose x differed from lag m's reference, [2m+1]: r
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int q = 0; q < 6; ++q) sm[m][q] = 0.0;
  // software pipeline, ICW_PF chunks deep: the loads of chunks i+1..i+ICW_PF are in flight
  // while chunk i is reduced (one wave per row: without it every chunk waits a full HBM
  // latency and only other waves hide it); the first ICW_PF were issued before step 1.
  // Two loops over the same pipeline: the first runs until every active lag has its shift
  // (usually chunk 0), the second -- the hot one -- carries no shift bookkeeping, so the
  // pair masks stay wave masks (no booleans materialised across the shift block).
  auto next = [&](int i0, double& x, uint32_t& rk, double (&r)[2]) {
    x = xq[0];
    rk = kq[0];
    r[0] = rq[0][0];
    r[1] = rq[0][1];
#pragma unroll
    for (int s = 0; s + 1 < ICW_PF; ++s) {   // rotate (register renames)
      xq[s] = xq[s + 1];
      kq[s] = kq[s + 1];
      rq[s][0] = rq[s + 1][0];
      rq[s][1] = rq[s + 1][1];
    }
    if (i0 + 64 * ICW_PF < An) load(i0 + 64 * ICW_PF, ICW_PF - 1);
  };
  // the pair rank 2k = RK minus the E correction of lag m.  Branch-free for both lags (a lag
  // without E entries reads empty blocks): the two lags' table reads issue
  // back to back and share one LDS latency.  The block's first two entries without a loop:
  // with ~1 NaN return per 6 rank blocks nearly every wave has a lane whose block holds
  // one, and a loop there made the whole wave run it (7.75 -> 7.30 ms at C2; a read past the
  // list end is masked, and the LDS region is padded by 2)
  auto pair_rank = [&](int m, uint32_t rk) {
    const uint64_t tb = T64[m][rk >> 6];
    const uint32_t lo = (uint32_t)tb, hi = (uint32_t)(tb >> 32);
    const uint32_t j0 = (lo & 0xffffu) >> 1, nj = lo >> 16, j1 = j0 + nj;
    const uint32_t e0 = hi & 0xffffu, e1 = hi >> 16;
    // absent entries are 0xffff, above every doubled rank: they count nothing
    int corr = (int)(lo & 0xffffu) + (e0 < rk ? 1 : 0) + (e0 <= rk ? 1 : 0) + (e1 < rk ? 1 : 0) + (e1 <= rk ? 1 : 0);
    for (uint32_t j = j0 + 2; j < j1; ++j) {   // a third entry or more (rare)
      const uint32_t e = eb[m][j];
      corr += (e < rk ? 1 : 0) + (e <= rk ? 1 : 0);
    }
    return rk - (uint32_t)corr;
  };
  auto accum = [&](int m, bool p, uint64_t bp, double x, uint32_t k2, double r) {
    // difference flags as wave masks: compares straight into scalar masks, ANDed with the
    // pair mask bp (a short-circuit p && ... would materialise the booleans in VGPRs)
    dm[2 * m] |= bp & __ballot(x != ax[m]);
    dm[2 * m + 1] |= bp & __ballot(r != ar[m]);
    if (!p) return;
    const double dx = x - ax[m], dy = r - ar[m];
    // the moment sums with fused multiply-adds: the records are tolerance-pinned (single-pass
    // moments about the first pair, ~1e-15 relative), not bit-pinned, and an fma per term is
    // both one instruction and one rounding fewer
    sm[m][0] += dx; sm[m][1] += dy;
    sm[m][2] = __builtin_fma(dx, dx, sm[m][2]);
    sm[m][3] = __builtin_fma(dy, dy, sm[m][3]);
    sm[m][4] = __builtin_fma(dx, dy, sm[m][4]);
    sm[m][5] = __builtin_fma((double)k2, dy, sm[m][5]);
    kk[m] += (uint64_t)k2 * k2;
  };
  // an inactive lag needs no shift (its records are never written)
  ref[0] = !act[0];
  ref[1] = !act[1];
  int i0 = 0;
  for (; i0 < An && !(ref[0] && ref[1]); i0 += 64) {
    double x, r[2];
    uint32_t rk;
    next(i0, x, rk, r);
    const uint32_t k2[2] = {pair_rank(0, rk), pair_rank(1, rk)};
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const bool p = (x == x) & (r[m] == r[m]);
      const uint64_t bp = __ballot(p);
      cnt[m] += __popcll(bp);
      if (!ref[m] && bp) {                    // wave-uniform: the first chunk with pairs
        const int l = __ffsll((unsigned long long)bp) - 1;
        ax[m] = fr_readlane_d(x, l);
        ar[m] = fr_readlane_d(r[m], l);
        ref[m] = true;
      }
      if (ref[m]) accum(m, p, bp, x, k2[m], r[m]);   // before the shift: no pairs to add
    }
  }
  for (; i0 < An; i0 += 64) {
    double x, r[2];
    uint32_t rk;
    next(i0, x, rk, r);
    const uint32_t k2[2] = {pair_rank(0, rk), pair_rank(1, rk)};
    const bool xo = x == x;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const bool p = xo & (r[m] == r[m]);
      const uint64_t bp = __ballot(p);
      cnt[m] += __popcll(bp);
      accum(m, p, bp, x, k2[m], r[m]);
    }
  }
  // 3. butterflies into the wave's scratch: [0,6) lag 0's sums, [6,12) lag 1's, [12,14) the
  // (2k)^2 sums (exact in doubles: < 2^53)
  double* sc = scr + wid * 32;
  {
    double a[16];
#pragma unroll
    for (int q = 0; q < 6; ++q) { a[q] = sm[0][q]; a[6 + q] = sm[1][q]; }
    a[12] = (double)kk[0];
    a[13] = (double)kk[1];
    a[14] = a[15] = 0.0;
    fr_part_bfly<16, false>(a, scr, 32, 0);
  }
  uint32_t dflags = 0;                        // wave OR of the difference bits
#pragma unroll
  for (int q = 0; q < 4; ++q) dflags |= (dm[q] != 0 ? 1u : 0u) << q;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (lane == 0) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      if (!act[m]) continue;
      const int64_t td = s + lagv[m];
      double* o = out + ((int64_t)(m * 4) * F + f) * D + td;
      const int64_t stp = F * D;
      const double nn = (double)cnt[m];
      double ic = qnan(), ric = qnan(), beta = qnan();
      if (cnt[m] >= 3) {
        const double* w = sc + 6 * m;
        const double sx = w[0], sy = w[1];
        const bool fconst = !((dflags >> (2 * m)) & 1), rconst = !((dflags >> (2 * m + 1)) & 1);
        if (!fconst && !rconst) {
          const double sxy = w[4] - sx * sy / nn;
          const double sxx = w[2] - sx * sx / nn;
          const double syy = w[3] - sy * sy / nn;
          // ranks: sum k = n(n+1)/2 (ties keep it), sum k^2 = sum (2k)^2 / 4: both exact
          const double skk = sc[12 + m] / 4.0 - nn * (nn + 1.0) * (nn + 1.0) / 4.0;
          const double sky = 0.5 * w[5] - 0.5 * (nn + 1.0) * sy;
          ic = fmin(1.0, fmax(-1.0, sxy / sqrt(sxx * syy)));
          ric = fmin(1.0, fmax(-1.0, sky / sqrt(skk * syy)));
        }
        // beta = sum x r / sum x^2 from the shifted sums
        const double a = ax[m], b = ar[m];
        const double sxx_raw = w[2] + 2.0 * a * sx + nn * a * a;
        const double sxr_raw = w[4] + a * sy + b * sx + nn * a * b;
        beta = sxx_raw > 0 ? sxr_raw / sxx_raw : qnan();
      }
      o[0] = nn;
      o[stp] = ic;
      o[2 * stp] = ric;
      o[3 * stp] = beta;
    }
  }
}


// Daily IC from the doubled ranks of the same panel: k_nan_positions, then k_ic_wave (one
// wave per row), then k_ic_ranked_list over the rows whose E lists were too long.
// work: [D][ICW_PC] positions, [D] counts, [1 + F*D] overflow list.  A <= 16384.
int64_t ic_ranked_work_len(int64_t F, int64_t D) { return D * (ICW_PC + 1) + 1 + F * D; }

fmx_status br_ic_ranked(const double* X, const fmx_rank2_t* RK, const double* R, int64_t F, int64_t D, int64_t A,
                        int64_t ld, const int32_t* lags_host, int n_lags, double* out, int32_t* work, hipStream_t st) {
  const int nt = 1024;
  const void* kl = FMX_EMAX_TABLE(k_ic_ranked_list)(nt, br_emax(A, nt));
  if (!kl) { set_error("row too long for the ranked IC kernels (A > 16384)"); return FMX_ERR_UNSUPPORTED; }
  if (F * D > 0x7fffffffll) { set_error("too many rows for one launch"); return FMX_ERR_UNSUPPORTED; }
  int32_t* pos = work;
  int32_t* npos = work + D * ICW_PC;
  int32_t* ovf = npos + D;
  k_nan_positions<<<(unsigned)((D + 3) / 4), 256, 0, st>>>(R, D, A, ld, pos, npos);
  FMX_LAUNCH_CHECK("k_nan_positions");
  static const int list_grid = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return 2 * std::max(cus, 1);              // two 1024-thread rows per CU
  }();
  const unsigned wave_grid = (unsigned)((F * D + ICW_WAVES - 1) / ICW_WAVES);
  for (int base = 0; base < n_lags; base += 2) {
    int NL = std::min(2, n_lags - base);
    int L0 = lags_host[base], L1 = NL > 1 ? lags_host[base + 1] : 0;
    double* o = out + (int64_t)base * 4 * F * D;
    k_ic_empty<<<(unsigned)F, 64, 0, st>>>(o, F, D, L0, L1, NL);
    FMX_LAUNCH_CHECK("k_ic_empty");
    FMX_HIP(hipMemsetAsync(ovf, 0, sizeof(int32_t), st));
    const int nbp = ((int)((2 * A) >> 6) + 2) & ~1;
    const size_t lds = sizeof(uint32_t) * (ICW_WAVES * 2 * (size_t)(2 * nbp + ICW_EC) + 2);
    k_ic_wave<<<wave_grid, 64 * ICW_WAVES, lds, st>>>(X, RK, R, F, D, A, ld, L0, L1, NL, o, pos, npos, ovf);
    FMX_LAUNCH_CHECK("k_ic_wave");
    void* args[] = {(void*)&X, (void*)&RK, (void*)&R, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&L0,
                    (void*)&L1, (void*)&NL, (void*)&o, (void*)&ovf};
    const unsigned g = (unsigned)std::min<int64_t>(F * D, list_grid);
    FMX_HIP(hipLaunchKernel(kl, dim3(g), dim3(nt), args, 0, st));
  }
  return FMX_OK;
}

// ------------------------------------------------------------------------------------
// The rank pass with the daily IC fused in (k_cs_rank_fa<..., IC>): cs_rank + cs_winsor
// (Yr, Yw set) or the ranks alone (both NULL: C5's IC rank pass), plus the two lags' IC
// records of every row, in one launch; the ranks never go to HBM.  Rows with more than
// FR_IC_EC NaN returns for a lag write their doubled ranks to RK and go through
// k_ic_ranked_list afterwards.

// NaN-return bits of every date: bits[d][w] bit b = R[d][32 w + b] is NaN (one wave per 64
// assets, ballot)
__global__ void __launch_bounds__(256)
k_nan_bits(const double* __restrict__ R, int64_t A, int64_t ld, int64_t nw, uint32_t* __restrict__ bits) {
  const int lane = threadIdx.x & 63;
  const int64_t i0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 64;
  if (i0 >= nw * 32) return;                  // whole waves
  const int64_t d = blockIdx.y, i = i0 + lane;
  const bool nan = i < A && !(R[d * ld + i] == R[d * ld + i]);
  const uint64_t b = __ballot(nan);
  if (lane == 0) {
    bits[d * nw + (i0 >> 5)] = (uint32_t)b;
    bits[d * nw + (i0 >> 5) + 1] = (uint32_t)(b >> 32);
  }
}

// Moment anchor of every date: its first non-NaN return (0 if none), one wave per date
__global__ void __launch_bounds__(64)
k_ret_anchor(const double* __restrict__ R, int64_t A, int64_t ld, double* __restrict__ rsh) {
  const int lane = threadIdx.x;
  const double* r = R + (int64_t)blockIdx.x * ld;
  double v = 0.0;
  for (int64_t i0 = 0; i0 < A; i0 += 64) {
    const double x = i0 + lane < A ? r[i0 + lane] : qnan();
    const uint64_t b = __ballot(x == x);
    if (b) {
      v = fr_readlane_d(x, __ffsll((unsigned long long)b) - 1);
      break;
    }
  }
  if (lane == 0) rsh[blockIdx.x] = v;
}

static int64_t nanb_words(int64_t A) { return (A + 63) / 64 * 2; }

// work (int32 units): rsh [D] doubles, NaN bits [D][nw], overflow list [1 + F*D]
int64_t rank_ic_work_len(int64_t F, int64_t D, int64_t A) { return 2 * D + D * nanb_words(A) + 1 + F * D; }

template <int NT, int E> constexpr auto kcrwi = k_cs_rank_fa<NT, E, false, true, true>;
template <int NT, int E> constexpr auto kcri = k_cs_rank_fa<NT, E, false, false, true>;

fmx_status br_cs_rank_winsor_ic(const double* X, double* Yr, double* Yw, const double* R, int64_t F, int64_t D,
                                int64_t A, int64_t ld, double qlo, double qhi, const int32_t* lags, int n_lags,
                                fmx_rank2_t* RK, int32_t* work, double* out, hipStream_t st) {
  const int nt_fa = fa_nt(A) == 1024 ? 1024 : 512;
  // the rank phase's keys / counters, then (IC tail) the exposures + E tables + partials
  const size_t lds_fr = std::max<size_t>({(size_t)A * 8, (size_t)FR_CS_WORDS * 4, (size_t)fr_ic_lds_bytes(A, nt_fa)});
  const int E = br_emax(A, nt_fa);
  const void* k = E < 0 ? nullptr : (Yr ? FMX_EMAX_TABLE(kcrwi)(nt_fa, E) : FMX_EMAX_TABLE(kcri)(nt_fa, E));
  const void* kl = FMX_EMAX_TABLE(k_ic_ranked_list)(1024, br_emax(A, 1024));
  if (!k || !kl || !lds_fits(k, lds_fr)) {
    set_error("fmx_cs_rank_winsor_ic: rows of A <= 16384 assets");
    return FMX_ERR_UNSUPPORTED;
  }
  if (F * D > 0x7fffffffll) { set_error("too many rows for one launch"); return FMX_ERR_UNSUPPORTED; }
  const int64_t nw = nanb_words(A);
  double* rsh = reinterpret_cast<double*>(work);              // work: 8-byte aligned device memory
  uint32_t* nanb = reinterpret_cast<uint32_t*>(work + 2 * D);
  int32_t* ovf = work + 2 * D + D * nw;
  k_nan_bits<<<dim3((unsigned)ceil_div(nw, 8), (unsigned)D), 256, 0, st>>>(R, A, ld, nw, nanb);
  FMX_LAUNCH_CHECK("k_nan_bits");
  k_ret_anchor<<<(unsigned)D, 64, 0, st>>>(R, A, ld, rsh);
  FMX_LAUNCH_CHECK("k_ret_anchor");
  int L0 = lags[0], L1 = n_lags > 1 ? lags[1] : 0, NL = n_lags;
  k_ic_empty<<<(unsigned)F, 64, 0, st>>>(out, F, D, L0, L1, NL);
  FMX_LAUNCH_CHECK("k_ic_empty");
  FMX_HIP(hipMemsetAsync(ovf, 0, sizeof(int32_t), st));
  FrIc ic{R, nanb, rsh, F, nw, L0, L1, NL, out, ovf, RK};
  FrZn zn{};
  int method = FMX_RANK_AVERAGE;
  const uint8_t* present = nullptr;
  fmx_rank2_t* RKrow = nullptr;
  // the IC tail's LDS (from 0) outlives the scan list behind the keys / counters
  const size_t loff = (size_t)fr_list_off(A, FR_CS_WORDS);
  const FrListLds ll = fr_list_lds(k, A, loff, lds_fr > loff ? lds_fr - loff : 0);
  int lcap = ll.cap;
  void* args[] = {(void*)&X, (void*)&Yr, (void*)&D, (void*)&A, (void*)&ld, (void*)&method, (void*)&present,
                  (void*)&Yw, (void*)&qlo, (void*)&qhi, (void*)&RKrow, (void*)&ic, (void*)&zn, (void*)&lcap};
  FMX_HIP(set_dyn_lds(k, ll.bytes));
  FMX_HIP(hipLaunchKernel(k, fmx_grid2(F, D), dim3(nt_fa), args, ll.bytes, st));   // date-major rows
  static const int list_grid = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      cus = 256;
    return 2 * std::max(cus, 1);
  }();
  const fmx_rank2_t* RKc = RK;
  void* largs[] = {(void*)&X, (void*)&RKc, (void*)&R, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&L0,
                   (void*)&L1, (void*)&NL, (void*)&out, (void*)&ovf};
  const unsigned g = (unsigned)std::min<int64_t>(F * D, list_grid);
  FMX_HIP(hipLaunchKernel(kl, dim3(g), dim3(1024), largs, 0, st));
  return FMX_OK;
}

}  // namespace fmx

BR_PHASE_EXPORT(fmx_debug_phase_ic)
