// Row operations on rows sorted in HBM: any row length up to 65,535 assets.
//
// * cs_rank, every method (operations.py:54-62: pandas Series.rank(method) over the
//   date's non-NaN rows, then (r - 1) / (len - 1) with len counting the NaN rows; a
//   single-row date -> 0.5; scipy 'average' with NaN propagation for the composites):
//   'first' / 'dense' past the LDS bitonic kernel's 8192 assets, every method past the
//   fine-bucket kernels' 16,384.
// * cs_winsor / cs_filter_center (operations.py:64-75) past 16,384: the order statistics
//   read off the sorted row.
// * group_rank_normalized (operations.py:152-168) for groups larger than the per-group LDS
//   sort takes (8192) or rows past 16,384: rows sorted by (group, value).
// * the daily IC / rank IC / beta (factor_selector.py:36-48) past 16,384 assets (where the
//   16-bit doubled ranks of the fine kernels end): ranks over each lag's pair-valid subset
//   read off the sorted row.
//
// keys = order-preserving u64 of the value (sentinel for NaN / absent cells), values = the
// asset index; rocPRIM's segmented radix sort (stable: equal keys keep ascending asset
// order = pandas 'first') sorts a chunk of rows, then one wave per row walks its sorted run
// (tie runs from ballots) and scatters the results.  Chunks of rows bound the workspace.
#include <rocprim/device/device_segmented_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include "rowkit.hpp"

namespace fmx {

constexpr int RS_NT = 256;
constexpr int64_t RS_CHUNK_ELEMS = (int64_t)1 << 26;   // sorted elements per chunk

struct RowStart {
  unsigned A;
  __host__ __device__ unsigned operator()(unsigned r) const { return r * A; }
};

typedef rocprim::transform_iterator<rocprim::counting_iterator<unsigned>, RowStart, unsigned> RowIter;

// keys / indices of rows [row0, row0 + gridDim.y), packed A per row
__global__ void __launch_bounds__(RS_NT)
k_rs_keys(const double* __restrict__ X, const uint8_t* __restrict__ present, int64_t D, int64_t A, int64_t ld,
          int64_t row0, uint64_t* __restrict__ keys, uint16_t* __restrict__ idx) {
  const int64_t a = (int64_t)blockIdx.x * RS_NT + threadIdx.x;
  if (a >= A) return;
  const int64_t r = blockIdx.y, row = row0 + r;
  const double v = X[row * ld + a];
  const bool p = present ? present[(row % D) * ld + a] != 0 : true;
  keys[r * A + a] = (p && v == v) ? okey(v) : KEY_SENTINEL;
  idx[r * A + a] = (uint16_t)a;
}

// ------------------------------------------------------------------------------------
// Ranks of one sorted segment by ONE wave: positions [b, b + n) of a sorted run whose keys
// (key_at(q), ascending, ties adjacent) are all valid; the element at sorted position q is
// asset idx_at(q) of the output row y.  Pass 1 (left to right, 64 positions per step) finds
// each position's tie-run start from the ballot of run starts below its lane (carried
// across steps) -- min / first / dense are final there; pass 2 (right to left) finds the
// run end for max / average.  y[asset] = half ? 0.5 : (rank - 1) / den.  Between the
// passes y holds the run start (exact in a double, read back by the same lane).
template <class KeyAt, class IdxAt>
__device__ void rs_wave_rank(KeyAt key_at, IdxAt idx_at, int64_t b, int64_t n, int method, bool half, double den,
                             double* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);   // lanes <= mine
  if (n <= 0) return;
  const bool need_end = method == FMX_RANK_MAX || method == FMX_RANK_AVERAGE ||
                        method == FMX_RANK_AVERAGE_PROPAGATE;
  int64_t carry_s = b, dense = 0;
  for (int64_t q0 = b; q0 < b + n; q0 += 64) {
    const int64_t q = q0 + lane;
    const bool in = q < b + n;
    const uint64_t k = in ? key_at(q) : KEY_SENTINEL;
    const uint64_t kp = (in && q > b) ? key_at(q - 1) : KEY_SENTINEL;
    const bool start = in && (q == b || k != kp);
    const uint64_t bal = __ballot(start);
    const uint64_t mine = bal & below;
    const int64_t s = mine ? q0 + 63 - __builtin_clzll(mine) : carry_s;
    const int64_t dr = dense + __popcll(mine);                  // distinct values <= mine
    if (in) {
      double r;
      const int64_t a = idx_at(q);
      if (method == FMX_RANK_FIRST) r = (double)(q - b + 1);
      else if (method == FMX_RANK_DENSE) r = (double)dr;
      else if (method == FMX_RANK_MIN) r = (double)(s - b + 1);
      else r = (double)s;                                       // run start, finished in pass 2
      y[a] = (need_end || half) ? r : (r - 1.0) / den;
    }
    if (bal) carry_s = q0 + 63 - __builtin_clzll(bal);
    dense += __popcll(bal);
  }
  if (!need_end && !half) return;
  __builtin_amdgcn_wave_barrier();
  int64_t carry_e = b + n;
  const int64_t last0 = b + ((n - 1) / 64) * 64;
  for (int64_t q0 = last0; q0 >= b; q0 -= 64) {
    const int64_t q = q0 + lane;
    const bool in = q < b + n;
    const uint64_t k = in ? key_at(q) : KEY_SENTINEL;
    const uint64_t kp = (in && q > b) ? key_at(q - 1) : KEY_SENTINEL;
    const bool start = in && (q == b || k != kp);
    const uint64_t bal = __ballot(start);
    const uint64_t above = bal & ~below;                        // run starts after my lane
    const int64_t e = above ? q0 + __builtin_ctzll(above) : carry_e;
    if (in) {
      const int64_t a = idx_at(q);
      double r;
      if (method == FMX_RANK_MAX) r = (double)(e - b);
      else if (method == FMX_RANK_AVERAGE || method == FMX_RANK_AVERAGE_PROPAGATE) {
        const int64_t s = (int64_t)y[a];                        // from pass 1 (same lane)
        r = (double)(s - b) + (double)(e - s + 1) / 2.0;        // #less + (#equal + 1) / 2
      } else {
        r = y[a];                                               // first / dense / min (half)
      }
      y[a] = half ? 0.5 : (r - 1.0) / den;
    }
    if (bal) carry_e = q0 + __builtin_ctzll(bal);
  }
}

// cs_rank of sorted rows (operations.py:54-62), every method: one wave per row.  Rows
// [row0, row0 + nr) of the chunk; keys sorted ascending per row (sentinel = NaN / absent,
// last), idx the assets.
constexpr int RS_WPB = 4;                     // rows (waves) per workgroup
__global__ void __launch_bounds__(64 * RS_WPB)
k_rs_rank(const uint64_t* __restrict__ keys, const uint16_t* __restrict__ idx, const double* __restrict__ X,
          const uint8_t* __restrict__ present, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld,
          int64_t row0, int64_t nr, int method) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * RS_WPB + (threadIdx.x >> 6);
  if (r >= nr) return;                        // whole waves
  const int64_t row = row0 + r;
  const uint64_t* k = keys + r * A;
  const uint16_t* ix = idx + r * A;
  const double* x = X + row * ld;
  double* y = Y + row * ld;
  const uint8_t* prow = present ? present + (row % D) * ld : nullptr;
  // nrow (present rows incl. NaN), nv (valid keys = first sentinel position)
  int64_t nrow = 0;
  for (int64_t i0 = 0; i0 < A; i0 += 64) {
    const int64_t i = i0 + lane;
    nrow += __popcll(__ballot(i < A && (prow ? prow[i] != 0 : true)));
  }
  int64_t lo = 0, hi = A;                     // first q with k[q] == sentinel
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (k[m] == KEY_SENTINEL) hi = m; else lo = m + 1;
  }
  const int64_t nv = lo;
  const bool prop = method == FMX_RANK_AVERAGE_PROPAGATE;
  const bool half = !prop && nrow == 1;
  const bool allnan = nv == 0 || (prop && nv < nrow);
  for (int64_t i0 = 0; i0 < A; i0 += 64) {    // absent -> NaN; NaN -> NaN (0.5 on a one-row date)
    const int64_t i = i0 + lane;
    if (i >= A) continue;
    const bool p = prow ? prow[i] != 0 : true;
    if (!p) y[i] = qnan();
    else if (!(x[i] == x[i])) y[i] = half ? 0.5 : qnan();
    else if (allnan) y[i] = half ? 0.5 : qnan();
  }
  if (allnan) return;
  __builtin_amdgcn_wave_barrier();
  rs_wave_rank([&](int64_t q) { return k[q]; }, [&](int64_t q) { return (int64_t)ix[q]; }, 0, nv, method, half,
               (double)(nrow - 1), y);
}

// cs_winsor (OP 0) / cs_filter_center (OP 1) of sorted rows (operations.py:64-75): the
// numpy 'linear' order statistics read straight off the sorted keys.  One wave per row.
template <int OP>
__global__ void __launch_bounds__(64 * RS_WPB)
k_rs_quantile(const uint64_t* __restrict__ keys, const double* __restrict__ X, const uint8_t* __restrict__ present,
              double* __restrict__ Y, int64_t D, int64_t A, int64_t ld, int64_t row0, int64_t nr, double qlo,
              double qhi) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * RS_WPB + (threadIdx.x >> 6);
  if (r >= nr) return;
  const int64_t row = row0 + r;
  const uint64_t* k = keys + r * A;
  const double* x = X + row * ld;
  double* y = Y + row * ld;
  const uint8_t* prow = present ? present + (row % D) * ld : nullptr;
  int64_t lo = 0, hi = A;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (k[m] == KEY_SENTINEL) hi = m; else lo = m + 1;
  }
  const int64_t nv = lo;
  double qv[2] = {qnan(), qnan()};
  if (nv > 0 && (OP == 1 || nv >= 5)) {
    const double qs[2] = {qlo, qhi};
#pragma unroll
    for (int z = 0; z < 2; ++z) {
      const double vi = (double)(nv - 1) * qs[z];
      int64_t k0, k1;
      double g;
      if (vi >= (double)(nv - 1)) {
        k0 = k1 = nv - 1;
        g = vi + 1.0;
      } else {
        const double pf = floor(vi);
        k0 = (int64_t)pf;
        k1 = k0 + 1;
        g = vi - pf;
      }
      const double a = okey_inv(k[k0]), b2 = okey_inv(k[k1]);
      const double diff = b2 - a;
      qv[z] = (g >= 0.5) ? b2 - diff * (1.0 - g) : a + diff * g;
    }
  }
  for (int64_t i0 = 0; i0 < A; i0 += 64) {
    const int64_t i = i0 + lane;
    if (i >= A) continue;
    const double v = x[i];
    double o;
    if (OP == 0) {
      o = v;
      if (nv >= 5) o = (v < qv[0]) ? qv[0] : ((v > qv[1]) ? qv[1] : v);
    } else {
      o = (v < qv[0] || v > qv[1]) ? v : 0.0;
    }
    y[i] = (prow && !prow[i]) ? qnan() : o;
  }
}

// group_rank_normalized of rows sorted by (group, value) (operations.py:152-168), any
// group size: one wave per row walks its groups (binary searches on the sorted group
// codes), ranks each group's non-NaN members with rs_wave_rank: (r - 1) / (n_valid - 1),
// n_valid <= 1 -> 0.5 for every member; NaN members -> NaN.  gkeys: sorted group codes
// (0xffffffff = no group / absent, last), idx: the assets.
__global__ void __launch_bounds__(64 * RS_WPB)
k_rs_group_rank(const uint32_t* __restrict__ gkeys, const uint16_t* __restrict__ idx, const double* __restrict__ X,
                double* __restrict__ Y, int64_t A, int64_t ld, int64_t row0, int64_t nr, int ngroups, int method) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * RS_WPB + (threadIdx.x >> 6);
  if (r >= nr) return;
  const int64_t row = row0 + r;
  const uint32_t* gk = gkeys + r * A;
  const uint16_t* ix = idx + r * A;
  const double* x = X + row * ld;
  double* y = Y + row * ld;
  for (int64_t i0 = 0; i0 < A; i0 += 64)      // members of no group (and absent cells): NaN
    if (i0 + lane < A && gk[i0 + lane] == 0xffffffffu) y[ix[i0 + lane]] = qnan();
  auto lower = [&](uint32_t g) {              // first position with code >= g
    int64_t lo = 0, hi = A;
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (gk[m] < g) lo = m + 1; else hi = m;
    }
    return lo;
  };
  int64_t gs = lower(0);
  for (int g = 0; g < ngroups; ++g) {
    const int64_t ge = lower((uint32_t)g + 1);
    if (ge > gs) {
      // members sorted by value, NaN (sentinel) ones last: n_valid = first NaN position
      int64_t lo = gs, hi = ge;
      while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        const double v = x[ix[m]];
        if (!(v == v)) hi = m; else lo = m + 1;
      }
      const int64_t nvg = lo - gs;
      for (int64_t q = lo + lane; q < ge; q += 64) y[ix[q]] = nvg <= 1 ? 0.5 : qnan();
      if (nvg <= 1) {
        for (int64_t q = gs + lane; q < lo; q += 64) y[ix[q]] = 0.5;
      } else {
        __builtin_amdgcn_wave_barrier();
        rs_wave_rank([&](int64_t q) { return okey(x[ix[q]]); }, [&](int64_t q) { return (int64_t)ix[q]; }, gs, nvg,
                     method, false, (double)(nvg - 1), y);
      }
    }
    gs = ge;
  }
}

// pass-2 keys of the group sort: the group code of each value-sorted element (no group,
// code out of range or absent -> 0xffffffff)
__global__ void __launch_bounds__(RS_NT)
k_rs_gkeys(const uint16_t* __restrict__ idx, const int32_t* __restrict__ G, const uint8_t* __restrict__ present,
           int64_t D, int64_t A, int64_t ld, int64_t row0, int ngroups, uint32_t* __restrict__ gk) {
  const int64_t q = (int64_t)blockIdx.x * RS_NT + threadIdx.x;
  if (q >= A) return;
  const int64_t r = blockIdx.y, row = row0 + r;
  const int64_t a = idx[r * A + q], d = row % D;
  const int32_t g = G[d * ld + a];
  const bool p = present ? present[d * ld + a] != 0 : true;
  gk[r * A + q] = (p && g >= 0 && g < ngroups) ? (uint32_t)g : 0xffffffffu;
}

// ------------------------------------------------------------------------------------
// Daily IC of sorted rows (factor_selector.py:36-48: pairs (X[f][s], R[s + L]) with both
// non-NaN, n < 3 -> NaN stats; IC = pearsonr(x, r), rank IC = pearsonr(rankdata(x over the
// pairs), r), beta = x.r / x.x), one wave per row (f, s) of the chunk.  Per lag:
//  pass 1 (left to right over the sorted valid keys): P(q) = # pairs at sorted positions < q
//    (ballot prefix); each position's tie-run start s_q; P(s_q) to scratch; the lag's moment
//    anchor = its first pair in sorted order;
//  pass 2 (right to left): the run end e_q (next run start), so a pair's doubled average rank
//    over the pairs is 2 * #less + #equal + 1 = P(s_q) + P(e_q) + 1; sums of x', r', x'^2,
//    r'^2, x'r' about the anchor, of 2k * r' and (2k)^2 (exact integers) -- the same
//    single-pass shifted moments and record formulas as k_ic_wave (~1e-15 relative to the
//    two-pass scipy arithmetic).
__device__ __forceinline__ double rs_wsum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ void __launch_bounds__(64 * RS_WPB)
k_rs_ic(const uint64_t* __restrict__ keys, const uint16_t* __restrict__ idx, uint32_t* __restrict__ scratch,
        const double* __restrict__ Rt, int64_t F, int64_t D, int64_t A, int64_t ld, int64_t row0, int64_t nr,
        int L0, int L1, int NL, double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * RS_WPB + (threadIdx.x >> 6);
  if (r >= nr) return;                        // whole waves
  const int64_t row = row0 + r, f = row / D, s = row % D;
  const uint64_t* k = keys + r * A;
  const uint16_t* ix = idx + r * A;
  uint32_t* Ps = scratch + r * A;
  int64_t lo = 0, hi = A;                     // nv = first sentinel position
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (k[m] == KEY_SENTINEL) hi = m; else lo = m + 1;
  }
  const int64_t nv = lo;
  const uint64_t below = (1ull << lane) - 1ull;        // lanes < mine
  const uint64_t incl = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
  for (int m = 0; m < NL; ++m) {
    const int64_t t = s + (m == 0 ? L0 : L1);
    if (t >= D) continue;                     // wave-uniform
    const double* rr = Rt + t * ld;
    // pass 1
    int64_t cnt = 0, carry_ps = 0;
    bool ref = false;
    double ax = 0.0, ar = 0.0;
    for (int64_t q0 = 0; q0 < nv; q0 += 64) {
      const int64_t q = q0 + lane;
      const bool in = q < nv;
      const uint64_t kq = in ? k[q] : KEY_SENTINEL;
      const uint64_t kp = (in && q > 0) ? k[q - 1] : KEY_SENTINEL;
      const double rv = in ? rr[ix[q]] : qnan();
      const bool pv = in && rv == rv;
      const bool start = in && (q == 0 || kq != kp);
      const uint64_t bs = __ballot(start), bp = __ballot(pv);
      const int64_t Pq = cnt + __popcll(bp & below);
      const uint64_t mine = bs & incl;
      const int sl = mine ? 63 - __builtin_clzll(mine) : 0;
      const int64_t sh = __shfl(Pq, sl, 64);
      if (in) Ps[q] = (uint32_t)(mine ? sh : carry_ps);
      if (bs) carry_ps = __shfl(Pq, 63 - __builtin_clzll(bs), 64);
      if (!ref && bp) {
        const int l = __ffsll((unsigned long long)bp) - 1;
        ax = __shfl(okey_inv(kq), l, 64);
        ar = __shfl(rv, l, 64);
        ref = true;
      }
      cnt += __popcll(bp);
    }
    __builtin_amdgcn_wave_barrier();
    // pass 2
    const int64_t tot = cnt;
    double sm[6] = {0, 0, 0, 0, 0, 0};
    double kk = 0.0;
    uint32_t dif = 0;
    int64_t carry_pe = tot, suf = 0;          // suf: pairs at positions >= the current chunk end
    if (tot >= 3) {
      for (int64_t q0 = ((nv - 1) / 64) * 64; q0 >= 0; q0 -= 64) {
        const int64_t q = q0 + lane;
        const bool in = q < nv;
        const uint64_t kq = in ? k[q] : KEY_SENTINEL;
        const uint64_t kp = (in && q > 0) ? k[q - 1] : KEY_SENTINEL;
        const double rv = in ? rr[ix[q]] : qnan();
        const bool pv = in && rv == rv;
        const bool start = in && (q == 0 || kq != kp);
        const uint64_t bs = __ballot(start), bp = __ballot(pv);
        const int64_t Pq = tot - (suf + __popcll(bp & ~below));     // pairs before q
        const uint64_t above = bs & ~incl;                          // run starts after my lane
        const int el = above ? __builtin_ctzll(above) : 0;
        const int64_t eh = __shfl(Pq, el, 64);
        const int64_t Pe = above ? eh : carry_pe;
        if (bs) carry_pe = __shfl(Pq, __builtin_ctzll(bs), 64);
        suf += __popcll(bp);
        if (pv) {
          const double x = okey_inv(kq);
          const double k2 = (double)((int64_t)Ps[q] + Pe + 1);
          const double dx = x - ax, dy = rv - ar;
          dif |= ((x != ax) ? 1u : 0u) | ((rv != ar) ? 2u : 0u);
          sm[0] += dx; sm[1] += dy;
          sm[2] += dx * dx; sm[3] += dy * dy; sm[4] += dx * dy;
          sm[5] += k2 * dy;
          kk += k2 * k2;                      // exact: < 2^53
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 6; ++q) sm[q] = rs_wsum(sm[q]);
    kk = rs_wsum(kk);
    const bool xvar = __ballot(dif & 1u) != 0, rvar = __ballot(dif & 2u) != 0;
    if (lane == 0) {
      double* o = out + ((int64_t)(m * 4) * F + f) * D + t;
      const int64_t stp = F * D;
      const double nn = (double)tot;
      double ic = qnan(), ric = qnan(), beta = qnan();
      if (tot >= 3) {
        const double sx = sm[0], sy = sm[1];
        if (xvar && rvar) {
          const double sxy = sm[4] - sx * sy / nn;
          const double sxx = sm[2] - sx * sx / nn;
          const double syy = sm[3] - sy * sy / nn;
          const double skk = kk / 4.0 - nn * (nn + 1.0) * (nn + 1.0) / 4.0;
          const double sky = 0.5 * sm[5] - 0.5 * (nn + 1.0) * sy;
          ic = fmin(1.0, fmax(-1.0, sxy / sqrt(sxx * syy)));
          ric = fmin(1.0, fmax(-1.0, sky / sqrt(skk * syy)));
        }
        const double sxx_raw = sm[2] + 2.0 * ax * sx + nn * ax * ax;
        const double sxr_raw = sm[4] + ax * sy + ar * sx + nn * ax * ar;
        beta = sxx_raw > 0 ? sxr_raw / sxx_raw : qnan();
      }
      o[0] = nn;
      o[stp] = ic;
      o[2 * stp] = ric;
      o[3 * stp] = beta;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// dates t < L get an empty record (n = 0, NaN stats)
__global__ void k_rs_ic_empty(double* out, int64_t F, int64_t D, int L, int m) {
  const int64_t f = blockIdx.x;
  for (int64_t td = threadIdx.x; td < min<int64_t>(L, D); td += blockDim.x) {
    double* o = out + ((int64_t)(m * 4) * F + f) * D + td;
    o[0] = 0.0;
    o[F * D] = qnan();
    o[2 * F * D] = qnan();
    o[3 * F * D] = qnan();
  }
}

static int64_t rs_chunk_rows(int64_t rows, int64_t A) {
  return std::max<int64_t>(1, std::min<int64_t>({rows, RS_CHUNK_ELEMS / std::max<int64_t>(A, 1), (int64_t)65535}));
}

static size_t rs_temp_bytes(int64_t crows, int64_t A) {
  size_t tb = 0;
  RowIter off(rocprim::counting_iterator<unsigned>(0), RowStart{(unsigned)A});
  (void)rocprim::segmented_radix_sort_pairs(nullptr, tb, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                      (const uint16_t*)nullptr, (uint16_t*)nullptr, (unsigned)(crows * A),
                                      (unsigned)crows, off, off + 1);
  return tb;
}

static size_t rs_temp_bytes32(int64_t crows, int64_t A) {
  size_t tb = 0;
  RowIter off(rocprim::counting_iterator<unsigned>(0), RowStart{(unsigned)A});
  (void)rocprim::segmented_radix_sort_pairs(nullptr, tb, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                      (const uint16_t*)nullptr, (uint16_t*)nullptr, (unsigned)(crows * A),
                                      (unsigned)crows, off, off + 1);
  return tb;
}

static int64_t al256(int64_t b) { return (b + 255) / 256 * 256; }

// Workspace of a chunk of cr rows: value keys in / out, asset indices in / out, the group
// keys in / out (group sort only) and the sort's temporary storage.
struct RsWork {
  uint64_t *kin, *kout;
  uint16_t *vin, *vout;
  uint32_t *gin, *gout;
  void* tmp;
  size_t tcap;
};

static int64_t rs_work_bytes(int64_t rows, int64_t A, bool groups) {
  const int64_t cr = rs_chunk_rows(rows, A), n = cr * A;
  int64_t b = 2 * al256(n * 8) + 2 * al256(n * 2);
  if (groups) b += 2 * al256(n * 4);
  const size_t t = groups ? std::max(rs_temp_bytes(cr, A), rs_temp_bytes32(cr, A)) : rs_temp_bytes(cr, A);
  return b + al256((int64_t)t);
}

static RsWork rs_carve(void* work, int64_t rows, int64_t A, bool groups) {
  const int64_t cr = rs_chunk_rows(rows, A), n = cr * A;
  char* w = static_cast<char*>(work);
  RsWork r{};
  r.kin = reinterpret_cast<uint64_t*>(w);
  w += al256(n * 8);
  r.kout = reinterpret_cast<uint64_t*>(w);
  w += al256(n * 8);
  r.vin = reinterpret_cast<uint16_t*>(w);
  w += al256(n * 2);
  r.vout = reinterpret_cast<uint16_t*>(w);
  w += al256(n * 2);
  if (groups) {
    r.gin = reinterpret_cast<uint32_t*>(w);
    w += al256(n * 4);
    r.gout = reinterpret_cast<uint32_t*>(w);
    w += al256(n * 4);
  }
  r.tmp = w;
  r.tcap = (size_t)(rs_work_bytes(rows, A, groups) - (w - static_cast<char*>(work)));
  return r;
}

// value keys of rows [r0, r0 + nr), sorted per row (stable: equal keys keep asset order)
static fmx_status rs_sort_chunk(const double* X, const uint8_t* present, int64_t D, int64_t A, int64_t ld, int64_t r0,
                                int64_t nr, RsWork& w, hipStream_t st) {
  k_rs_keys<<<dim3((unsigned)ceil_div(A, RS_NT), (unsigned)nr), RS_NT, 0, st>>>(X, present, D, A, ld, r0, w.kin,
                                                                                 w.vin);
  FMX_LAUNCH_CHECK("k_rs_keys");
  size_t tb = w.tcap;
  RowIter off(rocprim::counting_iterator<unsigned>(0), RowStart{(unsigned)A});
  FMX_HIP(rocprim::segmented_radix_sort_pairs(w.tmp, tb, w.kin, w.kout, w.vin, w.vout, (unsigned)(nr * A),
                                              (unsigned)nr, off, off + 1, 0, 64, st));
  return FMX_OK;
}

}  // namespace fmx

using namespace fmx;

extern "C" int64_t fmx_cs_rank_sorted_work_bytes(int64_t F, int64_t D, int64_t A) {
  if (F <= 0 || D <= 0 || A <= 0) return 0;
  return rs_work_bytes(F * D, A, false);
}

extern "C" fmx_status fmx_cs_rank_sorted(const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                                         int32_t method, const uint8_t* present, void* work, int64_t work_bytes,
                                         void* stream) {
  FMX_ARG(X && Y, "null panel");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  FMX_ARG(method >= FMX_RANK_AVERAGE && method <= FMX_RANK_AVERAGE_PROPAGATE, "unknown rank method");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  if (!work || work_bytes < fmx_cs_rank_sorted_work_bytes(F, D, A)) {
    set_error("workspace smaller than fmx_cs_rank_sorted_work_bytes()");
    return FMX_ERR_ARG;
  }
  hipStream_t st = as_stream(stream);
  const int64_t rows = F * D, cr = rs_chunk_rows(rows, A);
  RsWork w = rs_carve(work, rows, A, false);
  for (int64_t r0 = 0; r0 < rows; r0 += cr) {
    const int64_t nr = std::min(cr, rows - r0);
    fmx_status e = rs_sort_chunk(X, present, D, A, ld, r0, nr, w, st);
    if (e) return e;
    k_rs_rank<<<(unsigned)ceil_div(nr, RS_WPB), 64 * RS_WPB, 0, st>>>(w.kout, w.vout, X, present, Y, D, A, ld, r0, nr,
                                                                     method);
    FMX_LAUNCH_CHECK("k_rs_rank");
  }
  return FMX_OK;
}

extern "C" fmx_status fmx_cs_quantile_sorted(int32_t op, const double* X, double* Y, int64_t F, int64_t D, int64_t A,
                                             int64_t ld, double qlo, double qhi, const uint8_t* present, void* work,
                                             int64_t work_bytes, void* stream) {
  FMX_ARG(X && Y && Y != X, "null / aliased panel");
  FMX_ARG(op == 0 || op == 1, "op: 0 winsor, 1 filter_center");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  if (!work || work_bytes < fmx_cs_rank_sorted_work_bytes(F, D, A)) {
    set_error("workspace smaller than fmx_cs_rank_sorted_work_bytes()");
    return FMX_ERR_ARG;
  }
  hipStream_t st = as_stream(stream);
  const int64_t rows = F * D, cr = rs_chunk_rows(rows, A);
  RsWork w = rs_carve(work, rows, A, false);
  for (int64_t r0 = 0; r0 < rows; r0 += cr) {
    const int64_t nr = std::min(cr, rows - r0);
    fmx_status e = rs_sort_chunk(X, present, D, A, ld, r0, nr, w, st);
    if (e) return e;
    const void* k = op == 0 ? (const void*)k_rs_quantile<0> : (const void*)k_rs_quantile<1>;
    void* args[] = {(void*)&w.kout, (void*)&X, (void*)&present, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld,
                    (void*)&r0, (void*)&nr, (void*)&qlo, (void*)&qhi};
    FMX_HIP(hipLaunchKernel(k, dim3((unsigned)ceil_div(nr, RS_WPB)), dim3(64 * RS_WPB), args, 0, st));
  }
  return FMX_OK;
}

extern "C" int64_t fmx_group_rank_sorted_work_bytes(int64_t F, int64_t D, int64_t A) {
  if (F <= 0 || D <= 0 || A <= 0) return 0;
  return rs_work_bytes(F * D, A, true);
}

extern "C" int64_t fmx_ic_daily_sorted_work_bytes(int64_t F, int64_t D, int64_t A) {
  if (F <= 0 || D <= 0 || A <= 0) return 0;
  return rs_work_bytes(F * D, A, false);
}

extern "C" fmx_status fmx_ic_daily_sorted(const double* X, const double* R, int64_t F, int64_t D, int64_t A,
                                          int64_t ld, const int32_t* lags, int32_t n_lags, double* out, void* work,
                                          int64_t work_bytes, void* stream) {
  FMX_ARG(X && R && out && lags, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims (A <= 65535)");
  FMX_ARG(n_lags >= 1 && n_lags <= 8, "n_lags");
  for (int i = 0; i < n_lags; ++i) FMX_ARG(lags[i] >= 0, "lags must be >= 0");
  if (F == 0 || D == 0) return FMX_OK;
  if (!work || work_bytes < fmx_ic_daily_sorted_work_bytes(F, D, std::max<int64_t>(A, 1))) {
    set_error("workspace smaller than fmx_ic_daily_sorted_work_bytes()");
    return FMX_ERR_ARG;
  }
  hipStream_t st = as_stream(stream);
  for (int m = 0; m < n_lags; ++m) {
    k_rs_ic_empty<<<(unsigned)F, 64, 0, st>>>(out, F, D, lags[m], m);
    FMX_LAUNCH_CHECK("k_rs_ic_empty");
  }
  if (A == 0) return FMX_OK;
  const int64_t rows = F * D, cr = rs_chunk_rows(rows, A);
  RsWork w = rs_carve(work, rows, A, false);
  for (int64_t r0 = 0; r0 < rows; r0 += cr) {
    const int64_t nr = std::min(cr, rows - r0);
    fmx_status e = rs_sort_chunk(X, nullptr, D, A, ld, r0, nr, w, st);
    if (e) return e;
    uint32_t* scr = reinterpret_cast<uint32_t*>(w.kin);     // the sort's input keys are dead
    for (int base = 0; base < n_lags; base += 2) {
      const int NL = std::min(2, n_lags - base);
      const int L0 = lags[base], L1 = NL > 1 ? lags[base + 1] : 0;
      double* o = out + (int64_t)base * 4 * F * D;
      k_rs_ic<<<(unsigned)ceil_div(nr, RS_WPB), 64 * RS_WPB, 0, st>>>(w.kout, w.vout, scr, R, F, D, A, ld, r0, nr,
                                                                     L0, L1, NL, o);
      FMX_LAUNCH_CHECK("k_rs_ic");
    }
  }
  return FMX_OK;
}

extern "C" fmx_status fmx_group_rank_sorted(const double* X, const int32_t* G, double* Y, int64_t F, int64_t D,
                                            int64_t A, int64_t ld, int32_t ngroups, int32_t method,
                                            const uint8_t* present, void* work, int64_t work_bytes, void* stream) {
  FMX_ARG(X && G && Y && Y != X, "null / aliased panel");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  FMX_ARG(ngroups >= 0, "ngroups");
  FMX_ARG(method >= FMX_RANK_AVERAGE && method <= FMX_RANK_DENSE, "group rank methods average/min/max/first/dense");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  if (!work || work_bytes < fmx_group_rank_sorted_work_bytes(F, D, A)) {
    set_error("workspace smaller than fmx_group_rank_sorted_work_bytes()");
    return FMX_ERR_ARG;
  }
  hipStream_t st = as_stream(stream);
  const int64_t rows = F * D, cr = rs_chunk_rows(rows, A);
  RsWork w = rs_carve(work, rows, A, true);
  for (int64_t r0 = 0; r0 < rows; r0 += cr) {
    const int64_t nr = std::min(cr, rows - r0);
    // pass 1: by value (NaN last); pass 2 (stable): by group code -> groups in code order,
    // each group's members by value with its NaN members last
    fmx_status e = rs_sort_chunk(X, present, D, A, ld, r0, nr, w, st);
    if (e) return e;
    k_rs_gkeys<<<dim3((unsigned)ceil_div(A, RS_NT), (unsigned)nr), RS_NT, 0, st>>>(w.vout, G, present, D, A, ld, r0,
                                                                                    ngroups, w.gin);
    FMX_LAUNCH_CHECK("k_rs_gkeys");
    size_t tb = w.tcap;
    RowIter off(rocprim::counting_iterator<unsigned>(0), RowStart{(unsigned)A});
    FMX_HIP(rocprim::segmented_radix_sort_pairs(w.tmp, tb, w.gin, w.gout, w.vout, w.vin, (unsigned)(nr * A),
                                                (unsigned)nr, off, off + 1, 0, 32, st));
    k_rs_group_rank<<<(unsigned)ceil_div(nr, RS_WPB), 64 * RS_WPB, 0, st>>>(w.gout, w.vin, X, Y, A, ld, r0, nr,
                                                                           ngroups, method);
    FMX_LAUNCH_CHECK("k_rs_group_rank");
  }
  return FMX_OK;
}
