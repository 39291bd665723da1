// Factor x factor correlation GEMM (builder-defined).
//
// C = (sum_d Z_d^T Z_d) / (sum_d M_d^T M_d) where Z are per-date z-scored exposures
// (NaN -> 0) and M the 0/1 validity masks.  The reduction dimension K = dates x assets is
// huge (12.6e6 at 2520 x 5000) while F is 200..2000, so the output is cut into 128x128
// upper-triangular tiles x K-slices (date ranges):
//   * G = Z^T Z on fp64 MFMA (v_mfma_f64_16x16x4_f64), 512-thread workgroups (8 waves as
//     2 x 4, each a 64 x 32 sub-tile = 4 x 2 MFMA tiles), LDS-staged 128 x 32 fp64
//     chunks with the next chunk prefetched into registers while the MFMAs run.
//   * N = M^T M on bf16 MFMA (v_mfma_f32_32x32x16_bf16): 0/1 products are exact and the
//     fp32 accumulators stay exact while a slice holds < 2^24 (date, asset) pairs.
// The K-slices are reduced in a fixed order by k_gram_reduce (deterministic for any
// slice -> XCD placement).
#include <algorithm>
#include <type_traits>
#include <vector>

#include <cstdlib>

#include "exactsum.hpp"
#include "rowkit.hpp"

namespace fmx {

static_assert(EX_SLOTS == FMX_GRAM_EXACT_SLOTS, "exact Gram limb layout");

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef float flt16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef double dbl2 __attribute__((ext_vector_type(2)));

constexpr int GT = 128;        // output tile
constexpr int GK = 32;         // fp64 K chunk staged in LDS
constexpr int GKP = GK + 2;    // padded row: bank = (4 r + 2 k) mod 64, conflict-free ds_read_b64
constexpr int MK = 64;         // bf16 K chunk
constexpr int MKP = MK + 8;    // padded row (16 B)
constexpr size_t GRAM_F64_LDS = sizeof(double) * 2 * 2 * GT * GKP;   // k_gram_f64: 139 KB

// Tile t of the row-major upper triangle of an nb x nb tile grid: (0,0), (0,1), ...,
// (0,nb-1), (1,1), ...  (nb <= 16 at F = 2000, so the walk is short and block-uniform.)
__device__ __forceinline__ void upper_tile(int t, int nb, int& ti, int& tj) {
  ti = 0;
  while (t >= nb - ti) { t -= nb - ti; ++ti; }
  tj = ti + t;
}

// Workspace of the wide-panel Gram (fmx_gram): the per-slice partial tiles.
struct GramPlan {
  int nb;
  int64_t ntile, nslice, dps;
  int64_t part_elems() const { return nslice * ntile * GT * GT; }
};
static GramPlan gram_plan(int64_t F, int64_t A, int64_t d0, int64_t d1, bool mask) {
  GramPlan p;
  p.nb = (int)ceil_div(F, GT);
  p.ntile = (int64_t)p.nb * (p.nb + 1) / 2;
  const int64_t ndates = d1 - d0;
  // >= ~1024 workgroups to fill 256 CUs; bf16 slices must stay < 2^24 (date, asset) pairs
  p.nslice = std::max<int64_t>(1, std::min<int64_t>(ndates, ceil_div(1024, p.ntile)));
  p.dps = ceil_div(ndates, p.nslice);
  if (mask) {
    const int64_t cap = std::max<int64_t>(1, ((int64_t)1 << 24) / std::max<int64_t>(A, 1) - 1);
    p.dps = std::min(p.dps, cap);
  }
  p.nslice = ceil_div(ndates, p.dps);
  return p;
}

// per-date z-score of one (f, d) row; builder spec: mean/std(ddof=0) over non-NaN,
// NaN -> 0, sigma in {0, NaN} -> whole row 0 and M = 0.  M is written as bf16 0/1.
// Dates [d0, d0 + gridDim.x) of X [F][D][ld] into Z / M [F][Dout][ld] (Dout = the range
// length: a date chunk of a panel too large to materialise Z for all dates).  stats
// ([F][D] (mean, sd) of fmx_cs_moment_stats: numpy-pairwise, the oracle's moments bit for
// bit) when given; else block sums here (a constant row's sigma can then round to a tiny
// nonzero where numpy's is exactly 0).
__global__ void __launch_bounds__(256)
k_zscore_exposures(const double* __restrict__ X, const double* __restrict__ stats, double* __restrict__ Z,
                   uint16_t* __restrict__ M, int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t Dout) {
  __shared__ double dscr[16];
  const int64_t d = blockIdx.x, f = blockIdx.y;
  const double* x = X + (f * D + d0 + d) * ld;
  double* z = Z + (f * Dout + d) * ld;
  uint16_t* m = M + (f * Dout + d) * ld;
  double mean, sd;
  if (stats) {
    mean = stats[2 * (f * D + d0 + d)];
    sd = stats[2 * (f * D + d0 + d) + 1];
  } else {
    double s = 0.0, c = 0.0;
    for (int64_t a = threadIdx.x; a < A; a += 256) {
      double v = x[a];
      if (v == v) { s += v; c += 1.0; }
    }
    s = block_sum<256>(s, dscr);
    c = block_sum<256>(c, dscr);
    mean = c > 0 ? s / c : qnan();
    double q = 0.0;
    for (int64_t a = threadIdx.x; a < A; a += 256) {
      double v = x[a];
      if (v == v) q += (v - mean) * (v - mean);
    }
    q = block_sum<256>(q, dscr);
    sd = c > 0 ? sqrt(q / c) : qnan();
  }
  const bool ok = sd > 0.0;
  for (int64_t a = threadIdx.x; a < ld; a += 256) {
    double v = a < A ? x[a] : qnan();
    bool valid = ok && v == v;
    z[a] = valid ? (v - mean) / sd : 0.0;
    m[a] = valid ? (uint16_t)0x3f80 : (uint16_t)0;   // bf16 1.0 / 0.0
  }
}

// ---------------------------------------------------------------------------------------
// PADNAN: cells past the row / panel read as NaN (the direct Gram z-scores them to 0)
template <bool VEC, bool PADNAN = false>
__device__ __forceinline__ void load_chunk(const double* __restrict__ row, bool rowok, int64_t a0, int lc,
                                           int64_t A, double* r) {
  if (VEC && rowok && a0 + lc + 8 <= A) {
    const dbl2* p = reinterpret_cast<const dbl2*>(row + a0 + lc);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      dbl2 v = p[u];
      r[2 * u] = v[0];
      r[2 * u + 1] = v[1];
    }
  } else {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int64_t a = a0 + lc + u;
      r[u] = (rowok && a < A) ? row[a] : (PADNAN ? qnan() : 0.0);
    }
  }
}

// G = Z^T Z over one date slice, one 128 x 128 upper tile per workgroup: 8 waves as 2 x 4,
// each a 64 x 32 sub-tile of 4 x 2 fp64 16x16x4 MFMAs.  K = (date, 32-asset chunk) pairs;
// double-buffered LDS (2 x 2 x 128 x 34 doubles, dynamic): chunk c+1 is stored into the
// other buffer after chunk c's MFMAs and chunk c+2's loads go out right behind the one
// barrier per chunk, so the loads have a whole chunk of MFMAs to land.
template <bool VEC>
__global__ void __launch_bounds__(512)
k_gram_f64(const double* __restrict__ Z, int64_t F, int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t d1,
           int64_t dates_per_slice, int nb, int64_t ntile, double* __restrict__ part) {
  extern __shared__ double gsm[];             // [2][As | Bs], GT * GKP doubles each
  const int64_t tile = blockIdx.x, slice = blockIdx.y;
  int ti, tj;
  upper_tile((int)tile, nb, ti, tj);
  const int i0 = ti * GT, j0 = tj * GT;
  const int64_t ds = d0 + slice * dates_per_slice;
  const int64_t de = min<int64_t>(d1, ds + dates_per_slice);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  dbl4 acc[4][2];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[m][n] = dbl4{0.0, 0.0, 0.0, 0.0};
  const int lr = tid >> 2, lc = (tid & 3) * 8;   // 512 threads x 8 = 128 rows x 32 k
  const bool rowA = (i0 + lr) < F, rowB = (j0 + lr) < F;
  const int64_t nch = (A + GK - 1) / GK;
  const int64_t total = (de - ds) * nch;
  double ra[8], rb[8];
  auto issue = [&](int64_t c) {
    const int64_t d = ds + c / nch, a0 = (c % nch) * GK;
    load_chunk<VEC>(Z + ((int64_t)(i0 + lr) * D + d) * ld, rowA, a0, lc, A, ra);
    load_chunk<VEC>(Z + ((int64_t)(j0 + lr) * D + d) * ld, rowB, a0, lc, A, rb);
  };
  auto stage = [&](int buf) {
    double* As = gsm + buf * 2 * GT * GKP;
    double* Bs = As + GT * GKP;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      As[lr * GKP + lc + u] = ra[u];
      Bs[lr * GKP + lc + u] = rb[u];
    }
  };
  if (total > 0) {
    issue(0);
    stage(0);
  }
  __syncthreads();
  if (total > 1) issue(1);
  for (int64_t c = 0; c < total; ++c) {
    const double* As = gsm + (c & 1) * 2 * GT * GKP;
    const double* Bs = As + GT * GKP;
#pragma unroll
    for (int kk = 0; kk < GK; kk += 4) {
      const int k = kk + (lane >> 4);
      double af[4], bf[2];
#pragma unroll
      for (int m = 0; m < 4; ++m) af[m] = As[(wr * 64 + m * 16 + (lane & 15)) * GKP + k];
#pragma unroll
      for (int n = 0; n < 2; ++n) bf[n] = Bs[(wc * 32 + n * 16 + (lane & 15)) * GKP + k];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[m], bf[n], acc[m][n], 0, 0, 0);
    }
    if (c + 1 < total) stage((int)((c + 1) & 1));   // that buffer was last read in chunk c-1
    __syncthreads();
    if (c + 2 < total) issue(c + 2);
  }
  // C/D layout (f64 16x16x4): col = lane & 15, row = (lane >> 4) + 4 * reg
  double* p = part + (slice * ntile + tile) * (GT * GT);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 64 + m * 16 + (lane >> 4) + 4 * r;
        const int col = wc * 32 + n * 16 + (lane & 15);
        p[row * GT + col] = acc[m][n][r];
      }
}

// N = M^T M on bf16 MFMA.  256 threads = 4 waves as 2 x 2, each a 64 x 64 sub-tile of
// 2 x 2 v_mfma_f32_32x32x16_bf16 tiles.  Fragment maps (cdna_hip_programming.md sec. 3):
// lane l holds A[row l&31][k = 8(l>>5) + j], B[k][col l&31]; C col = l&31,
// row = (reg&3) + 8(reg>>2) + 4(l>>5).
__global__ void __launch_bounds__(256)
k_gram_mask(const uint16_t* __restrict__ M, int64_t F, int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t d1,
            int64_t dates_per_slice, int nb, int64_t ntile, double* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) uint16_t As[GT * MKP];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[GT * MKP];
  const int64_t tile = blockIdx.x, slice = blockIdx.y;
  int ti, tj;
  upper_tile((int)tile, nb, ti, tj);
  const int i0 = ti * GT, j0 = tj * GT;
  const int64_t ds = d0 + slice * dates_per_slice;
  const int64_t de = min<int64_t>(d1, ds + dates_per_slice);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  flt16 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.0f;
  // loader: 256 threads x 32 bf16 = 128 rows x 64 k
  const int lr = tid >> 1, lc = (tid & 1) * 32;
  const bool rowA = (i0 + lr) < F, rowB = (j0 + lr) < F;
  const bool vec = (ld % 8) == 0;   // 16-B aligned row segments
  // (date, 64-asset chunk) pairs flattened; the next chunk's loads are issued into
  // registers before this chunk's MFMAs (single-buffered LDS, as k_gram_f64)
  const int64_t nch = (A + MK - 1) / MK;
  const int64_t total = (de - ds) * nch;
  bf16x8 ra[4], rb[4];
  auto issue = [&](int64_t c) {
    const int64_t d = ds + c / nch, a0 = (c % nch) * MK;
    const uint16_t* ma = M + ((int64_t)(i0 + lr) * D + d) * ld;
    const uint16_t* mb = M + ((int64_t)(j0 + lr) * D + d) * ld;
    const bf16x8 za = {0, 0, 0, 0, 0, 0, 0, 0};
    if (vec && a0 + lc + 32 <= A) {
      const bf16x8* pa = reinterpret_cast<const bf16x8*>(ma + a0 + lc);
      const bf16x8* pb = reinterpret_cast<const bf16x8*>(mb + a0 + lc);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        ra[u] = rowA ? pa[u] : za;
        rb[u] = rowB ? pb[u] : za;
      }
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int64_t a = a0 + lc + 8 * u + e;
          ra[u][e] = (rowA && a < A) ? (short)ma[a] : (short)0;
          rb[u][e] = (rowB && a < A) ? (short)mb[a] : (short)0;
        }
    }
  };
  if (total > 0) issue(0);
  for (int64_t c = 0; c < total; ++c) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      *reinterpret_cast<bf16x8*>(&As[lr * MKP + lc + 8 * u]) = ra[u];
      *reinterpret_cast<bf16x8*>(&Bs[lr * MKP + lc + 8 * u]) = rb[u];
    }
    __syncthreads();
    if (c + 1 < total) issue(c + 1);
#pragma unroll
    for (int ks = 0; ks < MK; ks += 16) {
      const int k0 = ks + 8 * (lane >> 5);
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int m = 0; m < 2; ++m)
        af[m] = *reinterpret_cast<const bf16x8*>(&As[(wr * 64 + m * 32 + (lane & 31)) * MKP + k0]);
#pragma unroll
      for (int n = 0; n < 2; ++n)
        bfr[n] = *reinterpret_cast<const bf16x8*>(&Bs[(wc * 64 + n * 32 + (lane & 31)) * MKP + k0]);
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[m], bfr[n], acc[m][n], 0, 0, 0);
    }
    __syncthreads();
  }
  double* p = part + (slice * ntile + tile) * (GT * GT);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wr * 64 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = wc * 64 + n * 32 + (lane & 31);
        p[row * GT + col] = (double)acc[m][n][r];
      }
}

// Sum the slices in order and scatter the tile (and its mirror) into G[F][F].
// grid = (tile, GT*GT/256 element chunks).
__global__ void k_gram_reduce(const double* __restrict__ part, int64_t nslice, int64_t ntile, int nb, int64_t F,
                              double* __restrict__ G, int accumulate) {
  const int64_t tile = blockIdx.x;
  int ti, tj;
  upper_tile((int)tile, nb, ti, tj);
  const int i0 = ti * GT, j0 = tj * GT;
  {
    const int e = blockIdx.y * blockDim.x + threadIdx.x;
    if (e >= GT * GT) return;
    double s = 0.0;
    for (int64_t sl = 0; sl < nslice; ++sl) s += part[(sl * ntile + tile) * (GT * GT) + e];
    int i = i0 + e / GT, j = j0 + e % GT;
    if (i < F && j < F) {
      if (accumulate) s += G[(int64_t)i * F + j];
      G[(int64_t)i * F + j] = s;
      if (i0 != j0) G[(int64_t)j * F + i] = s;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Fused Gram for F <= 256: one workgroup per K-slice (a date range) computes the whole
// upper triangle of NB x NB 16x16 blocks (F padded to FP = 16 NB), reading the raw panel
// once.  Per K chunk (32 assets of one date) the 1024 threads load FP x 32 exposures,
// apply the z-score with the row stats (fmx_cs_moment_stats), and stage Z (fp64) and
// M (bf16 0/1) in LDS; each wave then runs the fp64 16x16x4 MFMAs (8 k-steps) and one
// bf16 16x16x32 MFMA of its triangle blocks (wave w owns triangle blocks w, w+16, ...).
// The next chunk's loads are in flight during the MFMAs.
constexpr int SG_NT = 1024;     // 16 waves: <= 6 triangle blocks per wave at F = 200
constexpr int SG_K = 32;          // assets per K chunk
constexpr int SG_KP = SG_K + 2;   // fp64 row pitch: conflict-free ds_read_b64 fragments
constexpr int SG_MP = SG_K + 8;   // bf16 row pitch: 16-B aligned rows

typedef float flt4 __attribute__((ext_vector_type(4)));

template <int NB, int MODE>   // MODE 0: G = Z Z^T on fp64 MFMA; 1: N = M M^T on bf16 MFMA
__global__ void __launch_bounds__(SG_NT)
k_gram_small(const double* __restrict__ X, const double* __restrict__ stats, int64_t F, int64_t D, int64_t A,
             int64_t ld, int64_t d0, int64_t d1, int64_t dps, double* __restrict__ part,
             uint32_t* __restrict__ mbits) {
  constexpr int FP = 16 * NB;
  constexpr int NTRI = NB * (NB + 1) / 2;
  constexpr int NWV = SG_NT / 64;
  constexpr int BPW = (NTRI + NWV - 1) / NWV;
  constexpr int NEL = FP * SG_K;              // elements per chunk
  constexpr int EPT = (NEL + SG_NT - 1) / SG_NT;   // loader elements per thread
  __shared__ double Zs[MODE == 0 ? FP * SG_KP : 1];
  __shared__ __attribute__((aligned(16))) uint16_t Ms[MODE == 1 ? FP * SG_MP : 8];
  __shared__ double mu_s[FP], sd_s[FP];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t slice = blockIdx.x;
  const int64_t ds = d0 + slice * dps;
  const int64_t de = min<int64_t>(d1, ds + dps);
  int blk[BPW];                                 // bi | bj << 8 (row-major triangle order), -1 = none
#pragma unroll
  for (int u = 0; u < BPW; ++u) {
    int j = wid + NWV * u, bi = 0;
    blk[u] = -1;
    if (j < NTRI) {
      while (j >= NB - bi) { j -= NB - bi; ++bi; }
      blk[u] = bi | ((bi + j) << 8);
    }
  }
  dbl4 gacc[MODE == 0 ? BPW : 1];
  flt4 nacc[MODE == 1 ? BPW : 1];
#pragma unroll
  for (int u = 0; u < (MODE == 0 ? BPW : 1); ++u) gacc[u] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int u = 0; u < (MODE == 1 ? BPW : 1); ++u) nacc[u] = flt4{0.0f, 0.0f, 0.0f, 0.0f};
  const int64_t nch = (A + SG_K - 1) / SG_K;
  const int64_t total = (de - ds) * nch;
  double xr[EPT];
  // chunk (date, asset block) walked by counters (no 64-bit divides in the loop)
  int64_t nd_iss = ds, na_iss = 0;               // next chunk to issue
  auto issue = [&]() {
    const int64_t d = nd_iss, a0 = na_iss * SG_K;
    if (++na_iss == nch) { na_iss = 0; ++nd_iss; }
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
      const int e = tid + SG_NT * u, r = e >> 5, cl = e & 31;
      const int64_t a = a0 + cl;
      xr[u] = (e < NEL && r < F && a < A) ? X[((int64_t)r * D + d) * ld + a] : qnan();
    }
  };
  auto load_stats = [&](int64_t d) {
    for (int r = tid; r < FP; r += SG_NT) {
      mu_s[r] = r < F ? stats[2 * ((int64_t)r * D + d)] : 0.0;
      sd_s[r] = r < F ? stats[2 * ((int64_t)r * D + d) + 1] : 0.0;
    }
  };
  if (total > 0) {
    issue();
    load_stats(ds);
  }
  // mask word of chunk c for row r: mword * F + r, word-major so that a chunk's rows are
  // one contiguous run (32-bit: F * dates * A/32 < 2^32)
  uint32_t mword = (uint32_t)((ds - d0) * nch);
  int64_t cin = 0, dcur = ds;                    // chunk c's asset block and date
  __syncthreads();
  for (int64_t c = 0; c < total; ++c) {
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
      const int e = tid + SG_NT * u, r = e >> 5, cl = e & 31;
      if (e >= NEL) continue;                   // wave-uniform (NEL is a multiple of 64)
      const double v = xr[u], sd = sd_s[r];
      const bool ok = (v == v) && (sd > 0.0);
      if (MODE == 0) Zs[r * SG_KP + cl] = ok ? (v - mu_s[r]) / sd : 0.0;
      else Ms[r * SG_MP + cl] = ok ? (uint16_t)0x3f80 : (uint16_t)0;   // bf16 1.0 / 0.0
      if (MODE == 0 && mbits) {
        // the chunk's validity bits, one 32-asset word per row (lanes 0-31: row r, 32-63:
        // row r+1): the pair counts N = M M^T come from these by AND + popcount
        const uint64_t bal = __ballot(ok);
        if ((lane & 31) == 0 && r < F) mbits[mword * (uint32_t)F + (uint32_t)r] = (uint32_t)(bal >> lane);
      }
    }
    __syncthreads();
    if (c + 1 < total) issue();
    if (MODE == 0) {
#pragma unroll 1
      for (int ks = 0; ks < SG_K; ks += 4) {     // not unrolled: bounds the fragment registers
        const int kk = ks + (lane >> 4);
#pragma unroll
        for (int u = 0; u < BPW; ++u) {
          if (blk[u] < 0) continue;               // wave-uniform
          const int bi = blk[u] & 0xff, bj = blk[u] >> 8;
          const double a = Zs[(bi * 16 + (lane & 15)) * SG_KP + kk];
          const double b = Zs[(bj * 16 + (lane & 15)) * SG_KP + kk];
          gacc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, gacc[u], 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < BPW; ++u) {
        if (blk[u] < 0) continue;
        const int bi = blk[u] & 0xff, bj = blk[u] >> 8;
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(&Ms[(bi * 16 + (lane & 15)) * SG_MP + 8 * (lane >> 4)]);
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(&Ms[(bj * 16 + (lane & 15)) * SG_MP + 8 * (lane >> 4)]);
        nacc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, nacc[u], 0, 0, 0);
      }
    }
    // the stats of chunk c were consumed before the barrier above
    if (c + 1 < total && ++cin == nch) { cin = 0; load_stats(++dcur); }
    ++mword;
    __syncthreads();
  }
  double* p = part + slice * (int64_t)FP * FP;
#pragma unroll
  for (int u = 0; u < BPW; ++u) {
    if (blk[u] < 0) continue;
    const int bi = blk[u] & 0xff, bj = blk[u] >> 8;
    const int col = bj * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (MODE == 0) p[(bi * 16 + (lane >> 4) + 4 * r) * FP + col] = gacc[u][r];             // f64 16x16x4 C map
      else p[(bi * 16 + 4 * (lane >> 4) + r) * FP + col] = (double)nacc[u & (MODE == 1 ? ~0 : 0)][r];  // bf16 16x16x32
    }
  }
}

// G = Z Z^T (fp64 MFMA) + validity bits, double-buffered: the k_gram_small<NB, 0> work
// with the chunk pipeline reorganised for MFMA occupancy.  k_gram_small's 57 KB of LDS let
// two workgroups share a CU, so the compiler capped it at 64 VGPRs and spilled the 6
// accumulator blocks (76 B/lane of scratch) and every chunk paid two barriers with the
// MFMA units idle while the whole workgroup z-scored the next chunk.  Here one workgroup
// owns a CU (amdgpu_waves_per_eu 4: 128 VGPRs, no spill), Zs is double-buffered, and each
// iteration stages chunk c+1 into the idle buffer (VALU + LDS writes, overlapping the other
// waves' MFMAs), issues the loads of chunk c+2, runs chunk c's MFMAs, then one barrier.
// Slices are equal ranges of the flattened (date, 32-asset block) chunk sequence, one per
// CU.  The row stats are double-buffered by date parity, loaded one date ahead.
//
// UNITS (the exact, GPU-count-independent Gram, fmx_gram_exact): the K range is cut into
// fixed units -- unit u = part u % S of date u / S, i.e. asset chunks [(u%S) nch / S,
// (u%S + 1) nch / S) of that date -- and each workgroup walks an equal range of units,
// writing its accumulators to part[unit][NTRI][256] at every unit boundary (dbl4 per lane,
// C-map order) and restarting them.  A unit's partial depends only on its own (date, asset
// range), never on the launch's date range or the CU count, so the exact fold of the
// partials (k_gram_fold) gives the same G however the dates are split over GPUs.
__host__ __device__ inline int64_t unit_chunk(int64_t u, int S, int64_t nch) {
  return (u / S) * nch + ((u % S) * nch) / S;
}

// k_gram_db: 16 waves (4 per SIMD, 128 registers each; 12 waves with 168: 12.97 vs 12.09 ms
// at C2 -- the fourth wave per SIMD hides more of the fragment reads than the registers buy)
#ifndef GDB_NT
#define GDB_NT 1024
#endif
#ifndef GDB_FENCE
#define GDB_FENCE 1
#endif
#ifndef GDB_PAD
#define GDB_PAD 1      // k_gram_db k-steps without the per-block branch (dummy block for short waves; 0: A/B arm, +0.4 ms at C2)
#endif
template <int NB, bool ZIN, bool UNITS = false>   // ZIN: X holds the z-scores (cs_zscore output), stats unused
__global__ void __launch_bounds__(GDB_NT) __attribute__((amdgpu_waves_per_eu(GDB_NT / 256, GDB_NT / 256)))
k_gram_db(const double* __restrict__ X, const double* __restrict__ stats, int64_t F, int64_t D, int64_t A,
          int64_t ld, int64_t d0, int64_t nch, int64_t total, int64_t nslice, double* __restrict__ part,
          uint32_t* __restrict__ mbits, int opt, int units_per_date = 1) {
  constexpr int FP = 16 * NB;
  constexpr int NTRI = NB * (NB + 1) / 2;
  constexpr int NWV = GDB_NT / 64;
  constexpr int BPW = (NTRI + NWV - 1) / NWV;
  constexpr int NEL = FP * SG_K;
  constexpr int EPT = (NEL + GDB_NT - 1) / GDB_NT;
  __shared__ double Zs[2][FP * SG_KP];
  __shared__ double mu_s[2][FP], sd_s[2][FP];
  // the wave index as a scalar: block ids, fragment rows and the A-row test in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t slice = blockIdx.x;
  // UNITS: ``total`` counts units; the slice's chunk range is its units' (contiguous) chunks
  const int S = units_per_date;
  const int64_t u0 = slice * total / nslice, u1 = (slice + 1) * total / nslice;
  const int64_t c0 = UNITS ? unit_chunk(u0, S, nch) : u0, c1 = UNITS ? unit_chunk(u1, S, nch) : u1;
  int64_t cur_u = u0, u_end = UNITS ? unit_chunk(u0 + 1, S, nch) : 0;
  // wave w owns the BPW consecutive triangle blocks [BPW w, BPW w + BPW) (row-major): most
  // of them share their block row, whose A fragment is then read once per k-step pair
  int blk[BPW];
#pragma unroll
  for (int u = 0; u < BPW; ++u) {
    int j = BPW * wid + u, bi = 0;
    blk[u] = -1;
    if (j < NTRI) {
      while (j >= NB - bi) { j -= NB - bi; ++bi; }
      blk[u] = bi | ((bi + j) << 8);
    }
  }
  dbl4 gacc[BPW];
#pragma unroll
  for (int u = 0; u < BPW; ++u) gacc[u] = dbl4{0.0, 0.0, 0.0, 0.0};
  double xr[EPT];
  // next chunk to load (date index relative to d0, asset block), walked by counters
  int64_t ld_d = c0 / nch, ld_a = c0 - (c0 / nch) * nch;
  // one 64-bit row address per issue, made opaque so the compiler cannot hoist the EPT
  // per-element row offsets out of the chunk loop (they spilled, and every reload's
  // vmcnt(0) wait serialised the chunk's loads); element u is GDB_NT / 32 rows further on
  auto issue = [&]() {
    const int64_t d = d0 + ld_d, a0 = ld_a * SG_K;
    if (++ld_a == nch) { ld_a = 0; ++ld_d; }
    const int r0 = tid >> 5, cl = tid & 31;
    const int64_t a = a0 + cl;
    const double* xb = X + ((int64_t)r0 * D + d) * ld + a;
    asm volatile("" : "+v"(xb));
    const int64_t step = (int64_t)(GDB_NT / 32) * D * ld;
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
      const int e = tid + GDB_NT * u, r = r0 + (GDB_NT / 32) * u;
      xr[u] = (e < NEL && r < F && a < A) ? xb[u * step] : qnan();
    }
  };
  auto load_stats = [&](int64_t dr) {             // date d0 + dr into buffer dr & 1
    if (ZIN) return;
    const int p = (int)(dr & 1);
    for (int r = tid; r < FP; r += GDB_NT) {
      mu_s[p][r] = r < F ? stats[2 * ((int64_t)r * D + d0 + dr)] : 0.0;
      sd_s[p][r] = r < F ? stats[2 * ((int64_t)r * D + d0 + dr) + 1] : 0.0;
    }
  };
  // stage the chunk held in xr (global chunk index c, date dr) into buffer b
  auto stage = [&](int64_t c, int64_t dr, int b) {
    const int p = (int)(dr & 1);
#pragma unroll
    for (int u = 0; u < EPT; ++u) {
      const int e = tid + GDB_NT * u, r = e >> 5, cl = e & 31;
      if (e >= NEL) continue;                     // wave-uniform (NEL is a multiple of 64)
      const double v = xr[u];
      bool ok;
      if (ZIN) {                                  // finite z-score; NaN / +-inf (sigma 0) -> invalid
        ok = (v - v) == 0.0;
        Zs[b][r * SG_KP + cl] = ok ? v : 0.0;
      } else {
        const double sd = sd_s[p][r];
        ok = (v == v) && (sd > 0.0);
        Zs[b][r * SG_KP + cl] = ok ? (v - mu_s[p][r]) / sd : 0.0;
      }
      const uint64_t bal = __ballot(ok);
      if ((lane & 31) == 0 && r < F) mbits[(uint32_t)c * (uint32_t)F + (uint32_t)r] = (uint32_t)(bal >> lane);
    }
  };
  if (c0 >= c1) return;
  // prologue: stats of the first chunk's date (and of the next chunk's, if it starts a
  // date), stage chunk c0, issue chunk c0 + 1
  int64_t cur_d = c0 / nch;                       // date (relative) of chunk c
  load_stats(cur_d);
  if (c0 + 1 < c1 && (c0 + 1) % nch == 0) load_stats(cur_d + 1);
  issue();
  __syncthreads();
  stage(c0, cur_d, 0);
  if (c0 + 1 < c1) issue();
  __syncthreads();
  // half the waves of each SIMD (waves s, s+4, s+8, s+12 share SIMD s) run their MFMAs
  // before staging the next chunk and half after, so the SIMD's MFMA pipe is not idle
  // while all four waves do the staging VALU work at the same time
  const bool mfma_first = (opt & 2) && ((wid >> 2) & 1);
  for (int64_t c = c0; c < c1; ++c) {
    const int b = (int)((c - c0) & 1);
    auto next = [&]() {
#ifdef GDB_DIAG_NOSTAGE
      return;                                     // diagnostic (wrong results): MFMAs only
#endif
      if (c + 1 < c1) {
        const int64_t dn = (c + 1) / nch;         // date of chunk c + 1
        stage(c + 1, dn, b ^ 1);                  // its stats were loaded a date ahead
        if (c + 2 < c1) {
          if ((c + 2) % nch == 0) load_stats(dn + 1);   // the buffer of date dn - 1: dead
          issue();
        }
      }
    };
    if (!mfma_first) next();
    // two k-steps per iteration: lane group g = lane >> 4 takes the chunk's k = ks + 2g and
    // ks + 2g + 1 in the two steps, so each fragment pair is ONE ds_read_b128 (the A and B
    // operands use the same k map, and every k of the chunk is taken once: the sum is the
    // same, only the MFMAs' accumulation order is fixed differently)
#pragma unroll 1
    for (int ks = 0; ks < SG_K; ks += 8) {
      const int kk = ks + 2 * (lane >> 4);
      int abi = -1;
      dbl2 a = dbl2{0.0, 0.0};
#pragma unroll
      for (int u = 0; u < BPW; ++u) {
#if GDB_PAD
        // no branch: a wave short of BPW blocks multiplies block (0, 0) -- which always
        // exists -- into the unused accumulator (never stored), so the k-step is
        // straight-line code (a wave owning no block at all, NTRI < waves, does the same)
        const int bk = blk[u] < 0 ? 0 : blk[u];
#else
        if (blk[u] < 0) continue;                 // wave-uniform
        const int bk = blk[u];
#endif
        const int bi = bk & 0xff, bj = bk >> 8;
        if (bi != abi) {                          // wave-uniform: a new block row
          a = *reinterpret_cast<const dbl2*>(&Zs[b][(bi * 16 + (lane & 15)) * SG_KP + kk]);
          abi = bi;
        }
        // (reading the next block's fragments ahead of these MFMAs: 12.67 vs 12.13 ms)
        const dbl2 bb = *reinterpret_cast<const dbl2*>(&Zs[b][(bj * 16 + (lane & 15)) * SG_KP + kk]);
        gacc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.x, bb.x, gacc[u], 0, 0, 0);
        gacc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a.y, bb.y, gacc[u], 0, 0, 0);
#if GDB_FENCE
        __builtin_amdgcn_sched_barrier(0);        // bounds the fragments in flight (VGPRs)
#endif
      }
    }
    if (UNITS) {
      while (c + 1 == u_end) {                    // unit cur_u complete (empty units: zeros)
        double* pu = part + (cur_u * NTRI) * 256 + lane * 4;
#pragma unroll
        for (int u = 0; u < BPW; ++u) {
          if (blk[u] < 0) continue;
          *reinterpret_cast<dbl4*>(pu + (int64_t)(BPW * wid + u) * 256) = gacc[u];
          gacc[u] = dbl4{0.0, 0.0, 0.0, 0.0};
        }
        if (++cur_u >= u1) break;
        u_end = unit_chunk(cur_u + 1, S, nch);
      }
    }
    if (mfma_first) next();
    __syncthreads();
  }
  if (UNITS) return;
  double* p = part + slice * (int64_t)FP * FP;
#pragma unroll
  for (int u = 0; u < BPW; ++u) {
    if (blk[u] < 0) continue;
    const int bi = blk[u] & 0xff, bj = blk[u] >> 8;
    const int col = bj * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) p[(bi * 16 + (lane >> 4) + 4 * r) * FP + col] = gacc[u][r];
  }
}

// Sum the slices in order (deterministic) for the upper-triangle blocks and mirror.
__global__ void k_gram_small_reduce(const double* __restrict__ partG, const double* __restrict__ partN,
                                    int64_t nslice, int FP, int64_t F, double* __restrict__ G,
                                    double* __restrict__ N, int accumulate,
                                    const unsigned long long* __restrict__ ncnt) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)FP * FP) return;
  const int i = (int)(e / FP), j = (int)(e % FP);
  if ((i >> 4) > (j >> 4) || i >= F || j >= F) return;
  const int64_t st = (int64_t)FP * FP;
  double g = 0.0, n = 0.0;
#pragma unroll 8
  for (int64_t sl = 0; sl < nslice; ++sl) {
    g += partG[sl * st + e];
    if (!ncnt) n += partN[sl * st + e];
  }
  if (ncnt) n = (double)ncnt[e];
  if (accumulate) {
    g += G[(int64_t)i * F + j];
    n += N[(int64_t)i * F + j];
  }
  G[(int64_t)i * F + j] = g;
  G[(int64_t)j * F + i] = g;
  N[(int64_t)i * F + j] = n;
  N[(int64_t)j * F + i] = n;
}

// Exact fold of k_gram_db<.,.,true>'s unit partials part[unit][NTRI][256] into the
// fixed-point limbs [EX_SLOTS][F][F] (upper triangle incl. the diagonal), and of the
// popcount pair counts into counts[F][F].  grid = (NTRI triangle blocks, unit groups) x
// 256 threads; thread e = element e of the block in the fp64 16x16x4 C map (lane e >> 2,
// register e & 3).  Each thread folds its group's units in registers, then adds its limbs
// with 64-bit integer atomics: integer addition, so neither the unit grouping nor the
// atomics' arrival order changes a bit of the result.
__global__ void __launch_bounds__(256)
k_gram_fold(const double* __restrict__ part, int64_t nunits, int64_t upg, int NB, int64_t F,
            int64_t* __restrict__ limbs, const unsigned long long* __restrict__ ncnt, int FP,
            int64_t* __restrict__ counts) {
  const int ntri = NB * (NB + 1) / 2;
  int t = blockIdx.x, bi = 0;
  while (t >= NB - bi) { t -= NB - bi; ++bi; }
  const int bj = bi + t;
  const int e = threadIdx.x, lane = e >> 2, r = e & 3;
  const int64_t row = bi * 16 + (lane >> 4) + 4 * r, col = bj * 16 + (lane & 15);
  if (row >= F || col >= F || row > col) return;
  int64_t acc[EX_SLOTS];
#pragma unroll
  for (int k = 0; k < EX_SLOTS; ++k) acc[k] = 0;
  const int64_t ua = (int64_t)blockIdx.y * upg, ub = min<int64_t>(nunits, ua + upg);
  const double* p = part + (int64_t)blockIdx.x * 256 + e;
#pragma unroll 4
  for (int64_t u = ua; u < ub; ++u) ex_add(acc, p[u * ntri * 256]);
  const int64_t FF = F * F, o = row * F + col;
#pragma unroll
  for (int k = 0; k < EX_SLOTS; ++k)
    if (acc[k]) atomicAdd(reinterpret_cast<unsigned long long*>(limbs + k * FF + o), (unsigned long long)acc[k]);
  if (blockIdx.y == 0 && ncnt) {
    const unsigned long long n = ncnt[row * FP + col];
    if (n) atomicAdd(reinterpret_cast<unsigned long long*>(counts + o), n);
  }
}

// G, N [F][F] (symmetric) from the (all-reduced) limbs and counts.
__global__ void __launch_bounds__(256)
k_gram_finalize(const int64_t* __restrict__ limbs, const int64_t* __restrict__ counts, int64_t F,
                double* __restrict__ G, double* __restrict__ N) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, FF = F * F;
  if (e >= FF) return;
  const int64_t i = e / F, j = e % F;
  if (i > j) return;
  int64_t acc[EX_SLOTS];
#pragma unroll
  for (int k = 0; k < EX_SLOTS; ++k) acc[k] = limbs[k * FF + e];
  const double g = ex_value(acc);
  G[e] = g;
  G[j * F + i] = g;
  if (N) {
    const double n = (double)counts[e];
    N[e] = n;
    N[j * F + i] = n;
  }
}

// N = M M^T from the validity bits k_gram_small<.,0> packed (32 assets per word, stored
// word-major [word][F]): one
// workgroup per (32 x 32 tile of the upper triangle, word range); 64-word chunks of the
// 64 rows staged in LDS, each thread owns one row i and four rows j.  Integer counts:
// exact, and order-free (64-bit atomics into ncnt[FP][FP]).
constexpr int PC_W = 64;
__global__ void __launch_bounds__(256)
k_gram_popc(const uint32_t* __restrict__ mbits, int64_t F, int64_t nw, int64_t wps, int FP,
            unsigned long long* __restrict__ ncnt) {
  __shared__ uint32_t Ai[32][PC_W + 1], Bj[32][PC_W + 1];
  const int tid = threadIdx.x;
  int tt = blockIdx.x, ti = 0;
  const int T = (int)((F + 31) / 32);
  while (tt >= T - ti) { tt -= T - ti; ++ti; }
  const int I0 = ti * 32, J0 = (ti + tt) * 32;
  const int64_t w0 = (int64_t)blockIdx.y * wps, w1 = min<int64_t>(nw, w0 + wps);
  const int i = tid >> 3, jg = tid & 7;
  unsigned acc[4] = {0u, 0u, 0u, 0u};
  for (int64_t wc = w0; wc < w1; wc += PC_W) {
    for (int q = tid; q < 32 * PC_W; q += 256) {
      const int r = q & 31, w = q >> 5;          // word-major bits: 32 rows of a word are contiguous
      const bool in = wc + w < w1;
      Ai[r][w] = (in && I0 + r < F) ? mbits[(wc + w) * F + I0 + r] : 0u;
      Bj[r][w] = (in && J0 + r < F) ? mbits[(wc + w) * F + J0 + r] : 0u;
    }
    __syncthreads();
#pragma unroll 8
    for (int w = 0; w < PC_W; ++w) {
      const uint32_t a = Ai[i][w];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += __popc(a & Bj[jg + 8 * k][w]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int gi = I0 + i, gj = J0 + jg + 8 * k;
    if (gi < F && gj < F && acc[k]) atomicAdd(&ncnt[(int64_t)gi * FP + gj], (unsigned long long)acc[k]);
  }
}

// Workspace of the fused F <= 256 Gram (fmx_gram_fused), carved from the caller's buffer:
// per-slice partial G tiles (and N tiles on the bf16-MFMA A/B path), the validity bits and
// the 64-bit pair counters.
struct SmallPlan {
  int64_t FP, nslice, dps, nw;
  bool mask_mfma;
  int64_t part_bytes() const { return (int64_t)sizeof(double) * FP * FP * nslice * (mask_mfma ? 2 : 1); }
  int64_t bits_bytes() const { return mask_mfma ? 0 : align256((int64_t)sizeof(uint32_t) * nw * FPF); }
  int64_t cnt_bytes() const { return mask_mfma ? 0 : (int64_t)sizeof(unsigned long long) * FP * FP; }
  int64_t bytes() const { return align256(part_bytes()) + bits_bytes() + cnt_bytes(); }
  int64_t FPF;   // F (rows of the bit matrix)
  static int64_t align256(int64_t b) { return (b + 255) / 256 * 256; }
};
static SmallPlan small_plan(int64_t F, int64_t A, int64_t d0, int64_t d1) {
  SmallPlan p;
  p.FP = 16 * ceil_div(std::max<int64_t>(F, 1), 16);
  p.FPF = F;
  const int64_t ndates = std::max<int64_t>(d1 - d0, 1);
  p.nslice = std::min<int64_t>(ndates, 512);
  p.dps = ceil_div(ndates, p.nslice);
  p.nslice = ceil_div(ndates, p.dps);
  // pair counts: validity bits packed by the fp64 pass + AND/popcount (default), or the
  // bf16 MFMA pass over the panel (FMX_GRAM_MASK_MFMA=1, kept for A/B)
  static const bool mask_mfma = getenv("FMX_GRAM_MASK_MFMA") != nullptr;
  p.mask_mfma = mask_mfma;
  p.nw = std::max<int64_t>(d1 - d0, 0) * ceil_div(A, (int64_t)SG_K);
  if (!mask_mfma) {
    // k_gram_db: one slice (workgroup) per CU over equal ranges of the nw chunks
    static const int cus = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n = 256;
      return std::max(n, 1);
    }();
    p.nslice = std::max<int64_t>(1, std::min<int64_t>(p.nw, cus));
    p.dps = 0;
  }
  return p;
}

}  // namespace fmx
// pair counts of k_gram_db's chunk-major validity bits (defined with k_gram_cnt_i8 below)
static fmx_status launch_pair_counts_cm(const uint32_t* mbits, int64_t F, int64_t nw, int FP,
                                        unsigned long long* ncnt, hipStream_t st);
namespace fmx {

template <int NB>
static fmx_status gram_small_launch(const double* X, const double* stats, double* G, double* N, int64_t F,
                                    int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t d1, int accumulate,
                                    char* work, hipStream_t st) {
  constexpr int FP = 16 * NB;
  const SmallPlan pl = small_plan(F, A, d0, d1);
  const int64_t nslice = pl.nslice, dps = pl.dps, nw = pl.nw;
  const int64_t st_elems = (int64_t)FP * FP * nslice;
  const bool mask_mfma = pl.mask_mfma;
  double* part = reinterpret_cast<double*>(work);
  uint32_t* mbits = mask_mfma ? nullptr : reinterpret_cast<uint32_t*>(work + SmallPlan::align256(pl.part_bytes()));
  unsigned long long* ncnt =
      mask_mfma ? nullptr
                : reinterpret_cast<unsigned long long*>(work + SmallPlan::align256(pl.part_bytes()) + pl.bits_bytes());
  if (ncnt) FMX_HIP(hipMemsetAsync(ncnt, 0, sizeof(unsigned long long) * FP * FP, st));
  static const bool db = getenv("FMX_GRAM_SINGLE_BUFFER") == nullptr;   // A/B switch
  if (!mask_mfma && db) {
    const int64_t nch = ceil_div(A, (int64_t)SG_K);
    // bit 1: MFMA / staging interleave across each SIMD's waves (default; A/B switch)
    static const int gopt = getenv("FMX_GRAM_OPT") ? atoi(getenv("FMX_GRAM_OPT")) : 2;
    if (stats)
      k_gram_db<NB, false><<<(unsigned)nslice, GDB_NT, 0, st>>>(X, stats, F, D, A, ld, d0, nch, nw, nslice, part,
                                                              mbits, gopt);
    else
      k_gram_db<NB, true><<<(unsigned)nslice, GDB_NT, 0, st>>>(X, stats, F, D, A, ld, d0, nch, nw, nslice, part,
                                                             mbits, gopt);
    FMX_LAUNCH_CHECK("k_gram_db");
  } else {
    if (!stats) { set_error("z-score input (stats == NULL) needs the default fused Gram path"); return FMX_ERR_UNSUPPORTED; }
    const int64_t dps2 = mask_mfma ? dps : ceil_div(d1 - d0, nslice);
    const int64_t ns2 = mask_mfma ? nslice : ceil_div(d1 - d0, dps2);
    k_gram_small<NB, 0><<<(unsigned)ns2, SG_NT, 0, st>>>(X, stats, F, D, A, ld, d0, d1, dps2, part, mbits);
    FMX_LAUNCH_CHECK("k_gram_small<G>");
    if (!mask_mfma && ns2 < nslice)   // fewer date slices than planned: zero the unused partials
      FMX_HIP(hipMemsetAsync(part + ns2 * FP * FP, 0, sizeof(double) * (nslice - ns2) * FP * FP, st));
  }
  if (mask_mfma) {
    k_gram_small<NB, 1><<<(unsigned)nslice, SG_NT, 0, st>>>(X, stats, F, D, A, ld, d0, d1, dps, part + st_elems,
                                                           nullptr);
    FMX_LAUNCH_CHECK("k_gram_small<N>");
  } else if (nw > 0) {
    if (fmx_status e = launch_pair_counts_cm(mbits, F, nw, FP, ncnt, st)) return e;
  }
  k_gram_small_reduce<<<(unsigned)ceil_div((int64_t)FP * FP, 256), 256, 0, st>>>(
      part, mask_mfma ? part + st_elems : nullptr, nslice, FP, F, G, N, accumulate, mask_mfma ? nullptr : ncnt);
  FMX_LAUNCH_CHECK("k_gram_small_reduce");
  return FMX_OK;
}

// Workspace of the exact Gram (fmx_gram_exact): unit partials, validity bits, pair counts.
// Units per date depend on A only (2560-asset halves of a 5,000-asset row), never on the
// date range or the device, so every GPU count folds the same partials.
struct ExactPlan {
  int64_t FP, ntri, nch, S, nunits, nw, F;
  int64_t part_bytes() const { return SmallPlan::align256((int64_t)sizeof(double) * nunits * ntri * 256); }
  int64_t bits_bytes() const { return SmallPlan::align256((int64_t)sizeof(uint32_t) * nw * F); }
  int64_t cnt_bytes() const { return (int64_t)sizeof(unsigned long long) * FP * FP; }
  int64_t bytes() const { return part_bytes() + bits_bytes() + cnt_bytes(); }
};
static int64_t exact_units_per_date(int64_t A) {
  const int64_t nch = std::max<int64_t>(1, ceil_div(A, (int64_t)SG_K));
  return std::min<int64_t>(nch, std::max<int64_t>(1, ceil_div(A, 2560)));
}
static ExactPlan exact_plan(int64_t F, int64_t A, int64_t d0, int64_t d1) {
  ExactPlan p;
  const int64_t nb = ceil_div(std::max<int64_t>(F, 1), 16);
  p.F = F;
  p.FP = 16 * nb;
  p.ntri = nb * (nb + 1) / 2;
  p.nch = ceil_div(A, (int64_t)SG_K);
  p.S = exact_units_per_date(A);
  p.nunits = std::max<int64_t>(d1 - d0, 0) * p.S;
  p.nw = std::max<int64_t>(d1 - d0, 0) * p.nch;
  return p;
}

template <int NB>
static fmx_status gram_exact_launch(const double* X, const double* stats, int64_t* limbs, int64_t* counts, int64_t F,
                                    int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t d1, char* work,
                                    hipStream_t st) {
  constexpr int FP = 16 * NB;
  const ExactPlan pl = exact_plan(F, A, d0, d1);
  if (pl.nunits == 0 || A == 0) return FMX_OK;
  FMX_ARG(pl.nw * F < ((int64_t)1 << 32), "panel too large for 32-bit validity-word indices");
  double* part = reinterpret_cast<double*>(work);
  uint32_t* mbits = reinterpret_cast<uint32_t*>(work + pl.part_bytes());
  unsigned long long* ncnt = reinterpret_cast<unsigned long long*>(work + pl.part_bytes() + pl.bits_bytes());
  FMX_HIP(hipMemsetAsync(ncnt, 0, pl.cnt_bytes(), st));
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return std::max(n, 1);
  }();
  const int64_t nslice = std::max<int64_t>(1, std::min<int64_t>(pl.nunits, cus));
  static const int gopt = getenv("FMX_GRAM_OPT") ? atoi(getenv("FMX_GRAM_OPT")) : 2;
  if (stats)
    k_gram_db<NB, false, true><<<(unsigned)nslice, GDB_NT, 0, st>>>(X, stats, F, D, A, ld, d0, pl.nch, pl.nunits,
                                                                    nslice, part, mbits, gopt, (int)pl.S);
  else
    k_gram_db<NB, true, true><<<(unsigned)nslice, GDB_NT, 0, st>>>(X, stats, F, D, A, ld, d0, pl.nch, pl.nunits,
                                                                   nslice, part, mbits, gopt, (int)pl.S);
  FMX_LAUNCH_CHECK("k_gram_db<units>");
  {
    const int64_t nw = pl.nw;
    if (fmx_status e = launch_pair_counts_cm(mbits, F, nw, FP, ncnt, st)) return e;
  }
  const int64_t ngroups = std::max<int64_t>(1, std::min<int64_t>(pl.nunits, 2048 / pl.ntri));
  const int64_t upg = ceil_div(pl.nunits, ngroups);
  k_gram_fold<<<dim3((unsigned)pl.ntri, (unsigned)ceil_div(pl.nunits, upg)), 256, 0, st>>>(
      part, pl.nunits, upg, NB, F, limbs, ncnt, FP, counts);
  FMX_LAUNCH_CHECK("k_gram_fold");
  return FMX_OK;
}

// ---------------------------------------------------------------------------------------
// Rolling correlation pruning (the builder-defined corr_prune selector, SURVEY A19, run for
// every processed day of FactorSelector): window j pools the per-date Gram partials of the
// raw dates [s0[j], s0[j] + W) -- the lag-1 factors of the window's dates -- and walks the
// day's metrics order (rank_IC_IR / IC_IR descending): a candidate above the threshold is
// kept iff |G(f,k) / N(f,k)| < rho for every kept k (0 where N = 0), up to top_x.  One
// wave per window; lane i sums the W partials of kept factor i in date order.
__global__ void __launch_bounds__(64)
k_window_prune(const double* __restrict__ partG, const double* __restrict__ partN, int FP, int64_t F, int64_t d_lo,
               int64_t nd, int W, const int32_t* __restrict__ s0, const int32_t* __restrict__ order,
               const double* __restrict__ metrics, int col, double thr, double rho, int top_x,
               double* __restrict__ w_out) {
  extern __shared__ int kept[];                   // [F]
  const int64_t j = blockIdx.x;
  const int lane = threadIdx.x;
  const int32_t* ord = order + j * F;
  const double* m = metrics + j * F * 8;
  const int64_t a0 = max<int64_t>((int64_t)s0[j], d_lo), a1 = min<int64_t>((int64_t)s0[j] + W, d_lo + nd);
  int nk = 0;
  for (int64_t pos = 0; pos < F && nk < top_x; ++pos) {
    const int f = ord[pos];
    const double v = m[(int64_t)f * 8 + col];
    if (!(v > thr)) continue;                     // NaN fails (factor_selection_methods.py:14 analogue)
    bool ok = true;
    for (int base = 0; base < nk && ok; base += 64) {
      bool bad = false;
      const int i = base + lane;
      if (i < nk) {
        const int k = kept[i];
        const int r = min(f, k), c = max(f, k);
        double g = 0.0, n = 0.0;
        for (int64_t d = a0; d < a1; ++d) {
          const int64_t off = (d - d_lo) * (int64_t)FP * FP + (int64_t)r * FP + c;
          g += partG[off];
          n += partN[off];
        }
        const double cc = n > 0.0 ? g / n : 0.0;
        bad = !(fabs(cc) < rho);
      }
      ok = __ballot(bad) == 0;
    }
    if (ok) {
      if (lane == 0) kept[nk] = f;
      ++nk;
      __syncthreads();
    }
  }
  double* w = w_out + j * F;
  for (int64_t f = lane; f < F; f += 64) w[f] = 0.0;
  __syncthreads();
  for (int i = lane; i < nk; i += 64) w[kept[i]] = 1.0 / (double)nk;
}

// The step's greedy prune over one correlation matrix (pipeline.run_step; the host walk of
// engine.greedy_prune restated): walk `order`; f is kept iff M(f) = max over the kept k of
// |C[f, k]| is NaN (a NaN propagates, as np.maximum does) or < rho; stop at top_x kept.
// One workgroup: M lives in LDS for every factor and absorbs row k of C (= column k: C is
// symmetric bit for bit) when k is kept, so each candidate costs one LDS read and a barrier,
// each kept one a coalesced row read.
constexpr int GP_NT = 1024;
__device__ __forceinline__ double gp_max(double a, double b) { return (a != a || b != b) ? qnan() : (a > b ? a : b); }
__global__ void __launch_bounds__(GP_NT)
k_greedy_prune(const double* __restrict__ C, int64_t F, int64_t ldc, const int64_t* __restrict__ order,
               int64_t n_order, double rho, int64_t top_x, int32_t* __restrict__ kept, int32_t* __restrict__ n_kept) {
  extern __shared__ double mx[];                 // [F]
  const int tid = threadIdx.x;
  for (int64_t f = tid; f < F; f += GP_NT) mx[f] = -__builtin_inf();
  __syncthreads();
  int64_t nk = 0;
  for (int64_t pos = 0; pos < n_order && nk < top_x; ++pos) {
    const int64_t c = order[pos];                // block-uniform
    if (c < 0 || c >= F) continue;
    const double m = mx[c];
    if (m == m && m >= rho) continue;            // every thread reads the same value
    if (tid == 0) kept[nk] = (int32_t)c;
    ++nk;
    __syncthreads();                             // all threads have read mx[c]
    const double* row = C + c * ldc;
    for (int64_t f = tid; f < F; f += GP_NT) mx[f] = gp_max(mx[f], fabs(row[f]));
    __syncthreads();
  }
  if (tid == 0) *n_kept = (int32_t)nk;
}

// Workspace of fmx_corr_prune_windows: per-date G and N partials over the dates the
// windows touch, then the window starts.
static void prune_dates(int64_t D, int64_t J, int W, const int32_t* s0_host, int64_t& d_lo, int64_t& nd) {
  d_lo = D;
  int64_t d_hi = 0;
  for (int64_t j = 0; j < J; ++j) {
    d_lo = std::min<int64_t>(d_lo, std::max<int64_t>(0, s0_host[j]));
    d_hi = std::max<int64_t>(d_hi, std::min<int64_t>(D, (int64_t)s0_host[j] + W));
  }
  if (d_hi <= d_lo) d_hi = d_lo = 0;
  nd = d_hi - d_lo;
}
static int64_t prune_part_bytes(int64_t F, int64_t nd) {
  const int64_t FP = 16 * ceil_div(std::max<int64_t>(F, 1), 16);
  return SmallPlan::align256((int64_t)sizeof(double) * 2 * std::max<int64_t>(nd, 1) * FP * FP);
}

template <int NB>
static fmx_status window_prune_launch(const double* X, const double* stats, int64_t F, int64_t D, int64_t A,
                                      int64_t ld, int64_t J, int W, const int32_t* s0_host, const int32_t* order,
                                      const double* metrics, int col, double thr, double rho, int top_x,
                                      double* w_out, char* work, hipStream_t st) {
  constexpr int FP = 16 * NB;
  int64_t d_lo, nd;
  prune_dates(D, J, W, s0_host, d_lo, nd);
  const int64_t d_hi = d_lo + nd;
  double* part = reinterpret_cast<double*>(work);
  int32_t* s0 = reinterpret_cast<int32_t*>(work + prune_part_bytes(F, nd));
  FMX_HIP(hipMemcpyAsync(s0, s0_host, sizeof(int32_t) * J, hipMemcpyHostToDevice, st));
  if (nd > 0) {
    // one slice per date: the partials ARE the per-date Grams (G on fp64 MFMA, N on bf16)
    k_gram_small<NB, 0><<<(unsigned)nd, SG_NT, 0, st>>>(X, stats, F, D, A, ld, d_lo, d_hi, 1, part, nullptr);
    FMX_LAUNCH_CHECK("k_gram_small<G>");
    k_gram_small<NB, 1><<<(unsigned)nd, SG_NT, 0, st>>>(X, stats, F, D, A, ld, d_lo, d_hi, 1,
                                                        part + nd * FP * FP, nullptr);
    FMX_LAUNCH_CHECK("k_gram_small<N>");
  }
  k_window_prune<<<(unsigned)J, 64, sizeof(int) * F, st>>>(part, part + nd * FP * FP, FP, F, d_lo, nd, W, s0, order,
                                                          metrics, col, thr, rho, top_x, w_out);
  FMX_LAUNCH_CHECK("k_window_prune");
  FMX_HIP(hipStreamSynchronize(st));              // s0_host may be a temporary
  return FMX_OK;
}

}  // namespace fmx

using namespace fmx;

static fmx_status check_work(const void* work, int64_t work_bytes, int64_t need, const char* query) {
  if (need > 0 && (!work || work_bytes < need)) {
    set_error(std::string("workspace smaller than ") + query + "()");
    return FMX_ERR_ARG;
  }
  return FMX_OK;
}

extern "C" int64_t fmx_gram_fused_work_bytes(int64_t F, int64_t D, int64_t A, int64_t d0, int64_t d1) {
  (void)D;
  if (F <= 0 || F > 256 || d1 <= d0) return 0;
  return small_plan(F, A, d0, d1).bytes();
}

extern "C" fmx_status fmx_gram_fused(const double* X, const double* stats, double* G, double* N, int64_t F,
                                     int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t d1, int32_t accumulate,
                                     void* work, int64_t work_bytes, void* stream) {
  FMX_ARG(X && G && N, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && d0 >= 0 && d1 <= D && d0 <= d1, "bad dims");
  if (F > 256) {
    set_error("fmx_gram_fused supports F <= 256; use fmx_zscore_exposures + fmx_gram");
    return FMX_ERR_UNSUPPORTED;
  }
  if (F == 0 || d1 == d0) return FMX_OK;
  if (fmx_status e = check_work(work, work_bytes, fmx_gram_fused_work_bytes(F, D, A, d0, d1),
                                "fmx_gram_fused_work_bytes"))
    return e;
  hipStream_t st = as_stream(stream);
  char* w = static_cast<char*>(work);
  const int nb = (int)ceil_div(F, 16);
  switch (nb) {
#define FMX_GS(K) \
  case K: return gram_small_launch<K>(X, stats, G, N, F, D, A, ld, d0, d1, accumulate, w, st);
    FMX_GS(1) FMX_GS(2) FMX_GS(3) FMX_GS(4) FMX_GS(5) FMX_GS(6) FMX_GS(7) FMX_GS(8)
    FMX_GS(9) FMX_GS(10) FMX_GS(11) FMX_GS(12) FMX_GS(13) FMX_GS(14) FMX_GS(15) FMX_GS(16)
#undef FMX_GS
    default: return FMX_ERR_UNSUPPORTED;
  }
}

extern "C" int64_t fmx_gram_exact_work_bytes(int64_t F, int64_t D, int64_t A, int64_t d0, int64_t d1) {
  (void)D;
  if (F <= 0 || F > 256 || d1 <= d0 || A <= 0) return 0;
  return exact_plan(F, A, d0, d1).bytes();
}

extern "C" fmx_status fmx_gram_exact(const double* X, const double* stats, int64_t* limbs, int64_t* counts,
                                     int64_t F, int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t d1,
                                     int32_t accumulate, void* work, int64_t work_bytes, void* stream) {
  FMX_ARG(X && limbs && counts, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && d0 >= 0 && d1 <= D && d0 <= d1, "bad dims");
  if (F > 256) {
    set_error("fmx_gram_exact supports F <= 256");
    return FMX_ERR_UNSUPPORTED;
  }
  hipStream_t st = as_stream(stream);
  if (!accumulate && F > 0) {
    FMX_HIP(hipMemsetAsync(limbs, 0, sizeof(int64_t) * FMX_GRAM_EXACT_SLOTS * F * F, st));
    FMX_HIP(hipMemsetAsync(counts, 0, sizeof(int64_t) * F * F, st));
  }
  if (F == 0 || d1 == d0 || A == 0) return FMX_OK;
  if (fmx_status e = check_work(work, work_bytes, fmx_gram_exact_work_bytes(F, D, A, d0, d1),
                                "fmx_gram_exact_work_bytes"))
    return e;
  char* w = static_cast<char*>(work);
  switch ((int)ceil_div(F, 16)) {
#define FMX_GE(K) \
  case K: return gram_exact_launch<K>(X, stats, limbs, counts, F, D, A, ld, d0, d1, w, st);
    FMX_GE(1) FMX_GE(2) FMX_GE(3) FMX_GE(4) FMX_GE(5) FMX_GE(6) FMX_GE(7) FMX_GE(8)
    FMX_GE(9) FMX_GE(10) FMX_GE(11) FMX_GE(12) FMX_GE(13) FMX_GE(14) FMX_GE(15) FMX_GE(16)
#undef FMX_GE
    default: return FMX_ERR_UNSUPPORTED;
  }
}

extern "C" fmx_status fmx_gram_exact_finalize(const int64_t* limbs, const int64_t* counts, double* G, double* N,
                                              int64_t F, void* stream) {
  FMX_ARG(limbs && G && (counts || !N), "null pointer");
  FMX_ARG(F >= 0, "bad dims");
  if (F == 0) return FMX_OK;
  k_gram_finalize<<<(unsigned)ceil_div(F * F, 256), 256, 0, as_stream(stream)>>>(limbs, counts, F, G, N);
  FMX_LAUNCH_CHECK("k_gram_finalize");
  return FMX_OK;
}

extern "C" int32_t fmx_gram_exact_units_per_date(int64_t A) { return (int32_t)exact_units_per_date(A); }

// Host run of the device's exact accumulator (exactsum.hpp is __host__ __device__): the CPU
// tests pin it against the numpy restatement without a GPU.
extern "C" void fmx_debug_exact_fold(const double* x, int64_t n, int64_t* limbs_out, double* value_out) {
  int64_t acc[EX_SLOTS] = {0, 0, 0, 0, 0, 0, 0};
  for (int64_t i = 0; i < n; ++i) ex_add(acc, x[i]);
  for (int k = 0; k < EX_SLOTS; ++k) limbs_out[k] = acc[k];
  if (value_out) *value_out = ex_value(acc);
}

extern "C" fmx_status fmx_zscore_exposures(const double* X, const double* stats, double* Z, uint16_t* M, int64_t F,
                                           int64_t D, int64_t A, int64_t ld, void* stream) {
  FMX_ARG(X && Z && M, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A, "bad dims");
  if (F == 0 || D == 0) return FMX_OK;
  k_zscore_exposures<<<dim3((unsigned)D, (unsigned)F), 256, 0, as_stream(stream)>>>(X, stats, Z, M, D, A, ld, 0, D);
  FMX_LAUNCH_CHECK("k_zscore_exposures");
  return FMX_OK;
}

extern "C" fmx_status fmx_zscore_exposures_range(const double* X, const double* stats, double* Z, uint16_t* M,
                                                 int64_t F, int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t d1,
                                                 void* stream) {
  FMX_ARG(X && Z && M, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && d0 >= 0 && d0 <= d1 && d1 <= D, "bad dims");
  if (F == 0 || d1 == d0) return FMX_OK;
  FMX_ARG(F <= 65535, "too many factors");
  k_zscore_exposures<<<dim3((unsigned)(d1 - d0), (unsigned)F), 256, 0, as_stream(stream)>>>(X, stats, Z, M, D, A,
                                                                                            ld, d0, d1 - d0);
  FMX_LAUNCH_CHECK("k_zscore_exposures");
  return FMX_OK;
}

static fmx_status gram_run(const void* Zp, bool mask, double* G, int64_t F, int64_t D, int64_t A, int64_t ld,
                           int64_t d0, int64_t d1, int accumulate, double* part, hipStream_t st) {
  const GramPlan pl = gram_plan(F, A, d0, d1, mask);
  dim3 grid((unsigned)pl.ntile, (unsigned)pl.nslice);
  if (mask) {
    k_gram_mask<<<grid, 256, 0, st>>>((const uint16_t*)Zp, F, D, A, ld, d0, d1, pl.dps, pl.nb, pl.ntile, part);
    FMX_LAUNCH_CHECK("k_gram_mask");
  } else if (ld % 2 == 0) {
    FMX_HIP(hipFuncSetAttribute((const void*)k_gram_f64<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GRAM_F64_LDS));
    k_gram_f64<true><<<grid, 512, GRAM_F64_LDS, st>>>((const double*)Zp, F, D, A, ld, d0, d1, pl.dps, pl.nb, pl.ntile, part);
    FMX_LAUNCH_CHECK("k_gram_f64");
  } else {
    FMX_HIP(hipFuncSetAttribute((const void*)k_gram_f64<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GRAM_F64_LDS));
    k_gram_f64<false><<<grid, 512, GRAM_F64_LDS, st>>>((const double*)Zp, F, D, A, ld, d0, d1, pl.dps, pl.nb, pl.ntile, part);
    FMX_LAUNCH_CHECK("k_gram_f64");
  }
  k_gram_reduce<<<dim3((unsigned)pl.ntile, GT * GT / 256), 256, 0, st>>>(part, pl.nslice, pl.ntile, pl.nb, F, G,
                                                                        accumulate);
  FMX_LAUNCH_CHECK("k_gram_reduce");
  return FMX_OK;
}

extern "C" int64_t fmx_gram_work_bytes(int64_t F, int64_t D, int64_t A, int64_t d0, int64_t d1, int32_t with_mask) {
  (void)D;
  if (F <= 0 || d1 <= d0) return 0;
  int64_t b = gram_plan(F, A, d0, d1, false).part_elems();
  if (with_mask) b = std::max(b, gram_plan(F, A, d0, d1, true).part_elems());
  return (int64_t)sizeof(double) * b;   // G then N reuse one partials buffer (stream-ordered)
}

extern "C" fmx_status fmx_gram(const double* Z, const uint16_t* M, double* G, double* N, int64_t F, int64_t D,
                               int64_t A, int64_t ld, int64_t d0, int64_t d1, int32_t accumulate, void* work,
                               int64_t work_bytes, void* stream) {
  FMX_ARG(Z && G, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && d0 >= 0 && d1 <= D && d0 <= d1, "bad dims");
  if (F == 0 || d1 == d0) return FMX_OK;
  const bool with_mask = M && N;
  if (fmx_status e = check_work(work, work_bytes, fmx_gram_work_bytes(F, D, A, d0, d1, with_mask),
                                "fmx_gram_work_bytes"))
    return e;
  hipStream_t st = as_stream(stream);
  double* part = static_cast<double*>(work);
  fmx_status e = gram_run(Z, false, G, F, D, A, ld, d0, d1, accumulate, part, st);
  if (e || !with_mask) return e;
  return gram_run(M, true, N, F, D, A, ld, d0, d1, accumulate, part, st);
}

// ---------------------------------------------------------------------------------------
// Wide-panel Gram straight from the panel (fmx_gram_direct, C4's 2000 x 2000): no Z / M
// materialisation.  The row moments are the caller's fmx_cs_moment_stats (numpy pairwise
// mean / std ddof=0: the oracle's z-score spec bit-for-bit, as the F <= 256 Gram uses).
// (1) validity bits (x not NaN, sigma > 0), factor-major [F][nd][nwd], written by the
// tile kernel's diagonal tiles while they stage (k_valid_bits: the standalone pass);
// (2) k_gram_f64w: G on fp64 MFMA with the z-score applied while a chunk is staged (X + the
// row's (mean, sd) instead of Z); (3) k_gram_popc_fm: N = M M^T as AND + popcount of the
// bits (exact integers), 64 x 64 tiles, 4 x 4 pairs per thread.
namespace fmx {

__global__ void __launch_bounds__(256)
k_valid_bits(const double* __restrict__ X, const double* __restrict__ stats, int64_t D, int64_t A, int64_t ld,
             int64_t d0, int64_t nd, int64_t nwd, uint32_t* __restrict__ bits) {
  const int64_t d = blockIdx.x, f = blockIdx.y;
  const double* x = X + (f * D + d0 + d) * ld;
  const bool ok = stats[2 * (f * D + d0 + d) + 1] > 0.0;     // sigma in {0, NaN}: no valid cell
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t* b = bits + (f * nd + d) * nwd;
  for (int64_t i0 = (int64_t)wid * 64; i0 < nwd * 32; i0 += 256) {
    const int64_t i = i0 + lane;
    const double v = x[i < A ? i : 0];
    const uint64_t bal = __ballot(ok && i < A && v == v);
    if (lane == 0) {
      b[i0 >> 5] = (uint32_t)bal;
      if ((i0 >> 5) + 1 < nwd) b[(i0 >> 5) + 1] = (uint32_t)(bal >> 32);
    }
  }
}

// Wide tiles for the direct Gram: 256 (i) x 128 (j) per workgroup, 16 waves as 4 x 4, each a
// 64 x 32 sub-tile of 4 x 2 fp64 16x16x4 MFMAs; K chunks of 16 assets, double-buffered LDS
// (2 x 384 x 18 doubles = 110 KB: one workgroup and four waves per SIMD per CU).  The
// z-score is applied while a chunk is staged, (x - mean) * (1 / sd) with the reciprocal once
// per row and chunk (dividing cost 86 ms of C4's Gram).  Measured against 128 x 128 tiles
// of 8 waves (profiles/r03/c4_gram_direct_ab.log): half the HBM fetch (65 vs 136 GB per
// launch at 252 dates) at the same time on one box -- the kernel is bound by the per-chunk
// load -> stage -> barrier chain, not by MFMA (skipping the below-diagonal blocks' MFMAs
// changed nothing) nor by HBM bandwidth.  Tile (bi, bj) covers rows [256 bi, +256),
// columns [128 bj, +128) for bj >= 2 bi: every (i <= j) pair lies in exactly one tile.
#ifndef GW_DIAG
#define GW_DIAG 0      // diagnostics (libfmx_d*.so only): 1 no panel loads, 2 no MFMAs, 3 no chunk barrier,
                       // 4 no z-score arithmetic while staging
#endif
constexpr int GW_I = 256, GW_J = 128, GW_K = 16, GW_KP = GW_K + 2;   // row pitch 36 dwords: conflict-free b64
constexpr size_t GRAM_W_LDS = sizeof(double) * 2 * (GW_I + GW_J) * GW_KP;
__host__ __device__ inline int64_t gw_ntile(int64_t F) {
  const int64_t nbi = (F + GW_I - 1) / GW_I, nbj = (F + GW_J - 1) / GW_J;
  int64_t n = 0;
  for (int64_t bi = 0; bi < nbi; ++bi) n += nbj - 2 * bi > 0 ? nbj - 2 * bi : 0;
  return n;
}
__device__ __forceinline__ void gw_tile(int t, int64_t F, int& bi, int& bj) {
  const int nbj = (int)((F + GW_J - 1) / GW_J);
  bi = 0;
  while (t >= nbj - 2 * bi) { t -= nbj - 2 * bi; ++bi; }
  bj = 2 * bi + t;
}

// ZC: X is the z pass's Zc chunk [F][nd][A] (z-scores, invalid -> 0, A a multiple of GW_K
// with zero pads): staged as loaded, no row stats, no validity bits.
template <bool VEC, bool ZC = false>
__global__ void __launch_bounds__(1024)
k_gram_f64w(const double* __restrict__ X, const double* __restrict__ zst, int64_t F, int64_t D, int64_t A, int64_t ld,
            int64_t d0, int64_t d1, int64_t dates_per_slice, int64_t phase, int64_t ntile, int64_t nslice, int xcd,
            int opt, double* __restrict__ part, uint16_t* __restrict__ bits16, int64_t nwd) {
  extern __shared__ double gsm[];             // [2][As (256 x KP) | Bs (128 x KP)]
  constexpr int BUF = (GW_I + GW_J) * GW_KP;
  // work item = slice * ntile + tile.  xcd: workgroups are dealt round-robin to the 8 XCDs,
  // so XCD x's k-th workgroup takes item x * per + k -- each XCD walks a contiguous run of
  // items (one date range, neighbouring tiles sharing row panels) and its L2 serves the
  // shared panels; else item = workgroup id.
  const int64_t total = ntile * nslice, wg = blockIdx.x + (int64_t)blockIdx.y * gridDim.x;
  int64_t item = wg;
  if (xcd == 1) {
    const int64_t per = (total + 7) / 8;
    item = (wg % 8) * per + wg / 8;
  }
  if (item >= total) return;                  // whole workgroup: before any barrier
  const int64_t tile = item % ntile, slice = item / ntile;
  int bi, bj;
  gw_tile((int)tile, F, bi, bj);
  const int i0 = bi * GW_I, j0 = bj * GW_J;
  // slice s: dates [d0 + s dps - phase, d0 + (s + 1) dps - phase) clipped to [d0, d1); a
  // nonzero phase aligns the slices to ABSOLUTE date blocks (fmx_gram_direct_exact)
  const int64_t ds = slice == 0 ? d0 : d0 + slice * dates_per_slice - phase;
  const int64_t de = min<int64_t>(d1, d0 + (slice + 1) * dates_per_slice - phase);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  dbl4 acc[4][2];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[m][n] = dbl4{0.0, 0.0, 0.0, 0.0};
  // loaders: A row tid >> 2 (4 assets at (tid & 3) * 4), B row tid >> 3 (2 assets at (tid & 7) * 2)
  const int ar = tid >> 2, ac = (tid & 3) * 4, br = tid >> 3, bc = (tid & 7) * 2;
  // 16 x 16 blocks this wave must compute (wave-uniform): not wholly below the diagonal
  // (i > j everywhere: never read) and not wholly past F -- a tile straddling the diagonal
  // skips the MFMAs of its lower half
  uint32_t live = 0;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int gi = i0 + wr * 64 + m * 16, gj = j0 + wc * 32 + n * 16;
      if (gi <= gj + 15 && gi < F && gj < F) live |= 1u << (m * 2 + n);
    }
  const bool rowA = (i0 + ar) < F, rowB = (j0 + br) < F;
  const int64_t nch = (A + GW_K - 1) / GW_K;
  const int64_t nchunk = (de - ds) * nch;
  double ra[4], rb[2];
  double2 sa, sb;                             // (mean, sd) of the staged rows' date
  // chunk cursors (wave-uniform) of the next issue and the next stage: chunks are issued and
  // staged in order, so (date, asset offset) advance by steps -- the c / nch, c % nch of a
  // 64-bit chunk index cost two long VALU division sequences per chunk
  int is_d = (int)ds, st_dr = (int)(ds - d0), st_j = 0, is_a = 0;
  const int nch32 = (int)nch;
  auto issue = [&](int64_t) {
    const int64_t d = is_d;
    const int a0 = is_a, A32 = (int)A;
    is_a += GW_K;
    if (is_a >= A) { is_a = 0; ++is_d; }
#if GW_DIAG == 1
    ra[0] = ra[1] = ra[2] = ra[3] = (double)(a0 & 7); rb[0] = rb[1] = (double)(d & 3);
    sa = make_double2(0.5, 1.0); sb = sa;
    return;
#endif
    // the row indices pass through an empty asm: the 64-bit row bases are recomputed per
    // chunk instead of being hoisted out of the chunk loop (their VGPRs would spill, and a
    // scratch reload waits on the prefetched chunk's loads)
    int rA = i0 + ar, rB = j0 + br;
    asm volatile("" : "+v"(rA), "+v"(rB));
    const double* pa = X + ((int64_t)rA * D + d) * ld + a0 + ac;
    const double* pb = X + ((int64_t)rB * D + d) * ld + a0 + bc;
    if (VEC && rowA && a0 + ac + 4 <= A32) {
      const dbl2 u = reinterpret_cast<const dbl2*>(pa)[0], v = reinterpret_cast<const dbl2*>(pa)[1];
      ra[0] = u[0]; ra[1] = u[1]; ra[2] = v[0]; ra[3] = v[1];
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) ra[q] = (rowA && a0 + ac + q < A32) ? pa[q] : qnan();
    }
    if (VEC && rowB && a0 + bc + 2 <= A32) {
      const dbl2 u = reinterpret_cast<const dbl2*>(pb)[0];
      rb[0] = u[0]; rb[1] = u[1];
    } else {
#pragma unroll
      for (int q = 0; q < 2; ++q) rb[q] = (rowB && a0 + bc + q < A32) ? pb[q] : qnan();
    }
    if constexpr (!ZC) {
      const double2* z = reinterpret_cast<const double2*>(zst);   // [F][D] (mean, 1/sd or 0)
      sa = rowA ? z[(int64_t)rA * D + d] : make_double2(0.0, 0.0);
      sb = rowB ? z[(int64_t)rB * D + d] : make_double2(0.0, 0.0);
    }
  };
  // validity bits: the diagonal tiles (bj = 2 bi, whose i-rows cover every row once per
  // date) write them while staging -- half-word (16 assets) per row and chunk, in the
  // factor-major [F][nd][2 nwd] u16 = [F][nd][nwd] u32 layout k_gram_popc_fm reads
  const bool wbits = bits16 != nullptr && bj == 2 * bi;
  auto stage = [&](int buf, int64_t) {
    double* As = gsm + buf * BUF;
    double* Bs = As + GW_I * GW_KP;
    const bool oka = !ZC && sa.y > 0.0, okb = !ZC && sb.y > 0.0;   // 1/sd > 0 <=> sd > 0
    if (!ZC && wbits) {                                      // workgroup-uniform
      // the row's 16 bits in (q, lane & 3) order: any asset order shared by every row
      // gives the same AND / popcount pair counts
      uint32_t hw = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint64_t m = __ballot(rowA && oka && ra[q] == ra[q]);
        hw |= (uint32_t)((m >> (lane & ~3)) & 0xfu) << (4 * q);
      }
      int rA = i0 + ar;
      asm volatile("" : "+v"(rA));                           // not hoisted: see issue()
      if ((lane & 3) == 0 && rowA) bits16[((int64_t)rA * (d1 - d0) + st_dr) * (2 * nwd) + st_j] = (uint16_t)hw;
    }
    if (++st_j == nch32) { st_j = 0; ++st_dr; }
    if constexpr (ZC) {
#pragma unroll
      for (int q = 0; q < 4; ++q) As[ar * GW_KP + ac + q] = rowA ? ra[q] : 0.0;
#pragma unroll
      for (int q = 0; q < 2; ++q) Bs[br * GW_KP + bc + q] = rowB ? rb[q] : 0.0;
      return;
    }
#if GW_DIAG == 4
#pragma unroll
    for (int q = 0; q < 4; ++q) As[ar * GW_KP + ac + q] = ra[q];
#pragma unroll
    for (int q = 0; q < 2; ++q) Bs[br * GW_KP + bc + q] = rb[q];
#else
#pragma unroll
    for (int q = 0; q < 4; ++q) As[ar * GW_KP + ac + q] = (oka && ra[q] == ra[q]) ? (ra[q] - sa.x) * sa.y : 0.0;
#pragma unroll
    for (int q = 0; q < 2; ++q) Bs[br * GW_KP + bc + q] = (okb && rb[q] == rb[q]) ? (rb[q] - sb.x) * sb.y : 0.0;
#endif
  };
  auto mfma_chunk = [&](int buf) {
    const double* As = gsm + buf * BUF;
    const double* Bs = As + GW_I * GW_KP;
#pragma unroll
    for (int kk = 0; kk < GW_K; kk += 4) {
      const int k = kk + (lane >> 4);
      double af[4], bf[2];
#pragma unroll
      for (int m = 0; m < 4; ++m) af[m] = As[(wr * 64 + m * 16 + (lane & 15)) * GW_KP + k];
#pragma unroll
      for (int n = 0; n < 2; ++n) bf[n] = Bs[(wc * 32 + n * 16 + (lane & 15)) * GW_KP + k];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          if ((live >> (m * 2 + n)) & 1u) {
#if GW_DIAG == 2
            acc[m][n][0] += af[m] * bf[n];
#else
            acc[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[m], bf[n], acc[m][n], 0, 0, 0);
#endif
          }
      // one k-step's fragments live at a time (the next step's reads are not hoisted over
      // these MFMAs): 128 VGPRs at four waves per SIMD without spilling
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  if (nchunk > 0) {
    issue(0);
    stage(0, 0);
  }
  __syncthreads();
  if (nchunk > 1) issue(1);
  // half the waves of each SIMD (waves s, s+4, s+8, s+12 share SIMD s) stage chunk c+1 and
  // issue chunk c+2's loads before their MFMAs of chunk c, half after: the SIMD's MFMA pipe
  // is fed while the other half does its staging VALU work and waits on its loads
  const bool stage_first = (opt & 1) && ((wid >> 2) & 1);
  for (int64_t c = 0; c < nchunk; ++c) {
    auto next = [&]() {
      if (c + 1 < nchunk) {
        stage((int)((c + 1) & 1), c + 1);     // that buffer was last read in chunk c-1
        if (c + 2 < nchunk) issue(c + 2);
      }
    };
    if (stage_first) next();
    mfma_chunk((int)(c & 1));
    if (!stage_first) next();
#if GW_DIAG == 3
    if (c < 2) __syncthreads();
#else
    __syncthreads();
#endif
  }
  double* p = part + (slice * ntile + tile) * (GW_I * GW_J);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 64 + m * 16 + (lane >> 4) + 4 * r;
        const int col = wc * 32 + n * 16 + (lane & 15);
        p[row * GW_J + col] = acc[m][n][r];
      }
}

// The Zc tile kernel with LDS-DMA staging (global_load_lds_dwordx4): the same 256 x 128 tiles,
// 16 waves of 64 x 32 sub-tiles and 16-asset chunks as k_gram_f64w<true, true>, but a chunk
// goes HBM -> LDS with no VGPRs and no staging instructions, three buffers deep: chunk c + 2
// is in flight while chunk c is multiplied, each wave retires its own DMA of chunk c + 1 with
// a counted vmcnt and one raw s_barrier per chunk publishes it to every wave.
// LDS image: 128-B rows (16 doubles), 16-B slot s of row r stored at slot s ^ ((r >> 1) & 7)
// -- the 16 rows one fragment read touches fall in 16 distinct 16-B positions of a bank row.
// A DMA wave-instruction fills 8 rows (1 KB); its lane L writes row 8q + (L >> 3), physical
// slot L & 7, so it loads the logical slot (L & 7) ^ ((row >> 1) & 7) from the row's chunk.
// Rows past F read row F - 1 (finite z-scores; their products land in rows / columns >= F,
// never folded).  Zc rows are [nd][A] contiguous: chunk c of a slice is 16 c doubles on.
#ifndef GZ_PF
#define GZ_PF 1        // fragment reads one k-step ahead of the MFMAs (0: A/B arm, 0.7 ms slower per 252 C4 dates)
#endif
#ifndef GZ_SGB
#define GZ_SGB 0       // A/B: the read / MFMA order of the prefetching k-loop pinned by sched_group_barrier
#endif
#ifndef GZ_PRIO
#define GZ_PRIO 0      // A/B: raised wave priority around each MFMA burst
#endif
constexpr int GZ_BUF = (GW_I + GW_J) * GW_K;                 // doubles per buffer (48 KB)
constexpr size_t GRAM_Z_LDS = sizeof(double) * 3 * GZ_BUF;     // 144 KB
// NW = 16: waves as 4 x 4 of 64 x 32 sub-tiles (4 x 2 MFMA blocks, 4 waves per SIMD);
// NW = 8: 4 x 2 of 64 x 64 (4 x 4 blocks: twice the MFMAs per fragment read, 2 waves per SIMD).
template <int NW>
__global__ void __launch_bounds__(NW * 64)
k_gram_zw(const double* __restrict__ Z, int64_t F, int64_t nd, int64_t A, int64_t dps, int64_t phase,
          int64_t ntile, int64_t nslice, double* __restrict__ part) {
  constexpr int WC = NW / 4, NBN = GW_J / WC / 16;           // wave columns, 16-blocks per wave row
  constexpr int PA = (GW_I / 8) / NW, PB = (GW_J / 8) / NW;  // DMA pieces per wave and chunk
  constexpr int NP = PA + PB;
  extern __shared__ double gsm[];
  const int64_t total = ntile * nslice, wg = blockIdx.x;
  const int64_t per = (total + 7) / 8;
  const int64_t item = (wg % 8) * per + wg / 8;    // XCD-contiguous runs of items, as k_gram_f64w
  if (item >= total) return;                       // whole workgroup: before any barrier
  const int64_t tile = item % ntile, slice = item / ntile;
  int bi, bj;
  gw_tile((int)tile, F, bi, bj);
  const int i0 = bi * GW_I, j0 = bj * GW_J;
  const int64_t ds = slice == 0 ? 0 : slice * dps - phase;
  const int64_t de = min<int64_t>(nd, (slice + 1) * dps - phase);
  const int64_t nchunk = (de - ds) * (A / GW_K);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WC, wc = wid % WC;
  dbl4 acc[4][NBN];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < NBN; ++n) acc[m][n] = dbl4{0.0, 0.0, 0.0, 0.0};
  uint32_t live = 0;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < NBN; ++n) {
      const int gi = i0 + wr * 64 + m * 16, gj = j0 + wc * (16 * NBN) + n * 16;
      if (gi <= gj + 15 && gi < F && gj < F) live |= 1u << (m * NBN + n);
    }
  constexpr uint32_t ALL = (1u << (4 * NBN)) - 1u;
  // this wave's DMA pieces per chunk: A row groups wid + NW q (rows 8 group + (L >> 3)), B
  // row groups wid + NW q; source pointers at the slice's first chunk
  const int lr = lane >> 3;
  auto src = [&](int lrow, int grow) -> const double* {
    const int r = min(grow, (int)F - 1);
    const int sl = (lane & 7) ^ ((lrow >> 1) & 7);
    return Z + ((int64_t)r * nd + ds) * A + 2 * sl;
  };
  const double* pp[NP];
#pragma unroll
  for (int q = 0; q < PA; ++q) pp[q] = src(8 * (wid + NW * q) + lr, i0 + 8 * (wid + NW * q) + lr);
#pragma unroll
  for (int q = 0; q < PB; ++q) pp[PA + q] = src(8 * (wid + NW * q) + lr, j0 + 8 * (wid + NW * q) + lr);
  auto dma = [&](int64_t c) {
#if GW_DIAG == 5 || GW_DIAG == 7
    return;                                          // diagnostics: no DMA (garbage operands)
#endif
    double* buf = gsm + (c % 3) * GZ_BUF;
    typedef __attribute__((address_space(3))) void lds_t;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int row = q < PA ? 8 * (wid + NW * q) : GW_I + 8 * (wid + NW * (q - PA));
      __builtin_amdgcn_global_load_lds((const void*)(pp[q] + c * GW_K), (lds_t*)(buf + row * GW_K), 16, 0, 0);
    }
  };
  auto wait_dma = [&](bool keep) {                 // keep: the newest chunk's NP pieces stay in flight
    if (keep) {
      if constexpr (NP == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };
  // fragment reads: row r (r & 15 = lane & 15), k = kk + g: logical slot k >> 1, half g & 1
  const int g = lane >> 4, r16 = lane & 15;
  if (nchunk > 0) dma(0);
  if (nchunk > 1) dma(1);
  wait_dma(nchunk > 1);
  __builtin_amdgcn_s_barrier();
  // waves whose 16 x 16 blocks are all live (all but the diagonal / edge tiles') run the
  // chunk loop without per-MFMA branches; both forms pass the same barriers
  auto run = [&](auto full) {
    for (int64_t c = 0; c < nchunk; ++c) {
      if (c + 2 < nchunk) dma(c + 2);               // buffer (c + 2) % 3 was last read in chunk c - 1
      const double* As = gsm + (c % 3) * GZ_BUF;
      const double* Bs = As + GW_I * GW_K;
      auto frag = [&](int kk, double* af, double* bf) {
        const int k = kk + g;
#if GW_DIAG == 6
#pragma unroll
        for (int m = 0; m < 4; ++m) af[m] = (double)(k + m);  // diagnostics: no LDS reads
#pragma unroll
        for (int n = 0; n < NBN; ++n) bf[n] = (double)(k - n);
        asm volatile("" : "+v"(af[0]), "+v"(bf[0]));
        return;
#endif
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const int row = wr * 64 + m * 16 + r16;
          af[m] = As[row * GW_K + (((k >> 1) ^ ((row >> 1) & 7)) << 1) + (k & 1)];
        }
#pragma unroll
        for (int n = 0; n < NBN; ++n) {
          const int row = wc * (16 * NBN) + n * 16 + r16;
          bf[n] = Bs[row * GW_K + (((k >> 1) ^ ((row >> 1) & 7)) << 1) + (k & 1)];
        }
      };
      auto mm = [&](const double* af, const double* bf) {
#if GZ_PRIO
        __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < NBN; ++n)
            if (decltype(full)::value || ((live >> (m * NBN + n)) & 1u))
              acc[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[m], bf[n], acc[m][n], 0, 0, 0);
#if GZ_PRIO
        __builtin_amdgcn_s_setprio(0);
#endif
      };
#if GZ_PF
      // next k-step's fragments are read before this step's MFMAs (two sets live)
      double af0[4], bf0[NBN], af1[4], bf1[NBN];
      frag(0, af0, bf0);
      frag(4, af1, bf1);
      mm(af0, bf0);
      frag(8, af0, bf0);
      mm(af1, bf1);
      frag(12, af1, bf1);
      mm(af0, bf0);
      mm(af1, bf1);
#if GZ_SGB
      if constexpr (decltype(full)::value) {
        // pin the order: reads of steps 0, 1 | MFMAs of 0 | reads of 2 | MFMAs of 1 | reads of
        // 3 | MFMAs of 2, 3 -- so each step's wait leaves the next step's reads in flight
        constexpr int RD = (4 + NBN) / 2, MF = 4 * NBN;     // ds_read2 per step, MFMAs per step
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * RD, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, MF, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, RD, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, MF, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, RD, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2 * MF, 0);
      }
#endif
#else
#pragma unroll
      for (int kk = 0; kk < GW_K; kk += 4) {
        double af[4], bf[NBN];
        frag(kk, af, bf);
        mm(af, bf);
        __builtin_amdgcn_sched_barrier(0);
      }
#endif
      wait_dma(c + 2 < nchunk);                     // chunk c + 1 landed (this wave's DMA)
#if GW_DIAG != 7
      __builtin_amdgcn_s_barrier();
#endif
    }
  };
  if (__builtin_amdgcn_readfirstlane(live) == ALL) run(std::true_type{});
  else run(std::false_type{});
  double* p = part + (slice * ntile + tile) * (GW_I * GW_J);
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < NBN; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wr * 64 + m * 16 + (lane >> 4) + 4 * r;
        const int col = wc * (16 * NBN) + n * 16 + (lane & 15);
        p[row * GW_J + col] = acc[m][n][r];
      }
}

// (mean, sd) -> (mean, 1/sd), 0 for sigma in {0, NaN}: the tile kernel's staging multiplies
__global__ void k_inv_stats(const double* stats, double* zi, int64_t n) {   // in place allowed
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const double m = stats[2 * e], sd = stats[2 * e + 1];
  zi[2 * e] = m;
  zi[2 * e + 1] = sd > 0.0 ? 1.0 / sd : 0.0;
}

// G from k_gram_f64w's slice partials: the pairs i <= j of each tile, summed over the
// slices in order (deterministic) and mirrored.
__global__ void k_gram_reduce_w(const double* __restrict__ part, int64_t nslice, int64_t ntile, int64_t F,
                                double* __restrict__ G, int accumulate) {
  const int64_t tile = blockIdx.x;
  int bi, bj;
  gw_tile((int)tile, F, bi, bj);
  const int e = blockIdx.y * blockDim.x + threadIdx.x;
  if (e >= GW_I * GW_J) return;
  const int64_t i = (int64_t)bi * GW_I + e / GW_J, j = (int64_t)bj * GW_J + e % GW_J;
  if (i > j || j >= F) return;
  double s = 0.0;
  for (int64_t sl = 0; sl < nslice; ++sl) s += part[(sl * ntile + tile) * (GW_I * GW_J) + e];
  if (accumulate) s += G[i * F + j];
  G[i * F + j] = s;
  G[j * F + i] = s;
}

// N[i][j] = sum over the bit words of popcount(bits[i] & bits[j]), factor-major bits
// [F][nw]: one workgroup per (64 x 64 upper tile, word range); 64-word chunks of the tile's
// 2 x 64 rows staged in LDS; thread (ty, tx) owns rows ty + 16 r and columns tx + 16 c
// (4 x 4 pairs: 8 LDS words per 16 AND/popcounts).  64-bit atomics into ncnt[F][F].
constexpr int PF_T = 64, PF_W = 64;
__global__ void __launch_bounds__(256)
k_gram_popc_fm(const uint32_t* __restrict__ bits, int64_t F, int64_t nw, int64_t wps,
               unsigned long long* __restrict__ ncnt) {
  __shared__ uint32_t Ai[PF_T][PF_W + 1], Bj[PF_T][PF_W + 1];
  const int tid = threadIdx.x;
  int tt = blockIdx.x, ti = 0;
  const int T = (int)((F + PF_T - 1) / PF_T);
  while (tt >= T - ti) { tt -= T - ti; ++ti; }
  const int I0 = ti * PF_T, J0 = (ti + tt) * PF_T;
  const int64_t w0 = (int64_t)blockIdx.y * wps, w1 = min<int64_t>(nw, w0 + wps);
  const int ty = tid >> 4, tx = tid & 15;
  unsigned acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = 0u;
  for (int64_t wc = w0; wc < w1; wc += PF_W) {
    for (int q = tid; q < PF_T * PF_W; q += 256) {
      const int r = q / PF_W, w = q % PF_W;     // row-contiguous words: coalesced
      const bool in = wc + w < w1;
      Ai[r][w] = (in && I0 + r < F) ? bits[(int64_t)(I0 + r) * nw + wc + w] : 0u;
      Bj[r][w] = (in && J0 + r < F) ? bits[(int64_t)(J0 + r) * nw + wc + w] : 0u;
    }
    __syncthreads();
#pragma unroll 4
    for (int w = 0; w < PF_W; ++w) {
      uint32_t a[4], b[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) a[r] = Ai[ty + 16 * r][w];
#pragma unroll
      for (int c = 0; c < 4; ++c) b[c] = Bj[tx + 16 * c][w];
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] += __popc(a[r] & b[c]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int gi = I0 + ty + 16 * r, gj = J0 + tx + 16 * c;
      if (gi < F && gj < F && gi <= gj && acc[r][c]) atomicAdd(&ncnt[(int64_t)gi * F + gj], (unsigned long long)acc[r][c]);
    }
}

// N = M M^T on the i8 matrix cores (v_mfma_i32_16x16x64_i8): the validity bits expand to 0/1
// bytes in registers, so the pair counts of a 64-bit K-step cost one MFMA per 16 x 16 block
// instead of 2 x 256 AND / popcounts.  128 x 128 upper tiles (incl. the diagonal) of 4 waves
// as 2 x 2, each a 64 x 64 sub-tile of 4 x 4 MFMAs (64 i32 accumulators per lane); chunks of
// 16 words per row staged in LDS.  Fragment map: lane (r = l & 15, g = l >> 4) of K-step s
// takes word 2s + (g >> 1) of its row, shifted by 4 (g & 1); dword q of its 16 operand bytes
// is (w >> q) & 0x01010101.  A and B lanes of one group hold the same k set on the MFMA's
// mirrored A / B maps, so every bit position meets its own in the other row exactly once
// whatever the hardware's k order within a group.  C/D: col = l & 15, row = 4 (l >> 4) + q.
constexpr int GC_T = 128, GC_KW = 16, GC_LP = 20;          // tile, words per chunk, LDS pitch
typedef int gc_v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ gc_v4i gc_expand(uint32_t t) {
  constexpr uint32_t M = 0x01010101u;
  gc_v4i d;
  d[0] = (int)(t & M);
  d[1] = (int)((t >> 1) & M);
  d[2] = (int)((t >> 2) & M);
  d[3] = (int)((t >> 3) & M);
  return d;
}
// CM: chunk-major bits [nw][F] (k_gram_db's mbits) instead of factor-major [F][nw]; ldn: the
// row stride of ncnt; btri: every pair of a 16 x 16 block on or above the block diagonal
// (k_gram_small_reduce / k_gram_fold's map) instead of the pairs i <= j.
template <bool VEC, bool CM = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4)))
k_gram_cnt_i8(const uint32_t* __restrict__ bits, int64_t F, int64_t nw, int64_t wps,
              unsigned long long* __restrict__ ncnt, int64_t ldn = 0, int btri = 0) {
  __shared__ uint32_t Ls[2 * GC_T * GC_LP];                   // rows 0..127: I tile, 128..255: J
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int tt = blockIdx.x, ti = 0;
  const int T = (int)((F + GC_T - 1) / GC_T);
  while (tt >= T - ti) { tt -= T - ti; ++ti; }
  const int I0 = ti * GC_T, J0 = (ti + tt) * GC_T;
  const int64_t w0 = (int64_t)blockIdx.y * wps, w1 = min<int64_t>(nw, w0 + wps);
  const int wr = wid >> 1, wc = wid & 1, r = lane & 15, g = lane >> 4;
  const int hw = g >> 1, sh = 4 * (g & 1);
  gc_v4i acc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = gc_v4i{0, 0, 0, 0};
  // loader: thread t stages words 4 (t & 3) .. +3 of rows (t >> 2) + 64 i, i = 0..3
  const int lr = tid >> 2, lw = (tid & 3) * 4;
  for (int64_t wc0 = w0; wc0 < w1; wc0 += GC_KW) {
    uint32_t v[4][4];
    if constexpr (CM) {
      // thread t: row t of the 256 (I then J), the chunk's 16 words (a word's rows are contiguous)
      const int64_t fr = tid < GC_T ? I0 + tid : J0 + tid - GC_T;
      const bool ok = fr < F;
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q >> 2][q & 3] = (ok && wc0 + q < w1) ? bits[(wc0 + q) * F + fr] : 0u;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = lr + 64 * i;
        const int64_t fr = row < GC_T ? I0 + row : J0 + row - GC_T;
        const uint32_t* p = bits + fr * nw + wc0 + lw;
        const bool ok = fr < F;
        if (VEC && ok && wc0 + lw + 4 <= w1) {
          const uint4 u = *reinterpret_cast<const uint4*>(p);
          v[i][0] = u.x; v[i][1] = u.y; v[i][2] = u.z; v[i][3] = u.w;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[i][q] = (ok && wc0 + lw + q < w1) ? p[q] : 0u;
        }
      }
    }
    __syncthreads();                                          // the previous chunk's reads are done
    if constexpr (CM) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<uint4*>(&Ls[tid * GC_LP + 4 * i]) = make_uint4(v[i][0], v[i][1], v[i][2], v[i][3]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<uint4*>(&Ls[(lr + 64 * i) * GC_LP + lw]) = make_uint4(v[i][0], v[i][1], v[i][2], v[i][3]);
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < GC_KW / 2; ++s) {
      gc_v4i a[4], b[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) a[m] = gc_expand(Ls[(wr * 64 + m * 16 + r) * GC_LP + 2 * s + hw] >> sh);
#pragma unroll
      for (int n = 0; n < 4; ++n) b[n] = gc_expand(Ls[(GC_T + wc * 64 + n * 16 + r) * GC_LP + 2 * s + hw] >> sh);
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[m], b[n], acc[m][n], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);                      // one K-step's fragments live at a time
    }
  }
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gi = I0 + wr * 64 + m * 16 + 4 * g + q, gj = J0 + wc * 64 + n * 16 + r;
        const int c = acc[m][n][q];
        const bool up = btri ? (gi >> 4) <= (gj >> 4) : gi <= gj;
        if (gi < F && gj < F && up && c) atomicAdd(&ncnt[(int64_t)gi * (ldn ? ldn : F) + gj], (unsigned long long)c);
      }
}

// N from the counts (upper triangle incl. the diagonal), mirrored; accumulate adds to N
__global__ void k_gram_counts(const unsigned long long* __restrict__ ncnt, int64_t F, double* __restrict__ N,
                              int accumulate) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= F * F) return;
  const int64_t i = e / F, j = e % F;
  if (i > j) return;
  double n = (double)ncnt[e];
  if (accumulate) n += N[i * F + j];
  N[i * F + j] = n;
  N[j * F + i] = n;
}

// Exact fold of k_gram_f64w's block partials (fmx_gram_direct_exact): element e of tile
// `tile` (i <= j < F) adds its nslice partials into fixed-point limbs in registers (ex_add)
// and stores / adds them to limbs [EX_SLOTS][F][F]; its pair count from ncnt likewise.  Every
// (i <= j) lies in exactly one tile: one writer per element, no atomics.
__global__ void __launch_bounds__(256)
k_gram_fold_w(const double* __restrict__ part, int64_t nslice, int64_t ntile, int64_t F,
              const unsigned long long* __restrict__ ncnt, int64_t* __restrict__ limbs,
              int64_t* __restrict__ counts, int accumulate) {
  const int64_t tile = blockIdx.x;
  int bi, bj;
  gw_tile((int)tile, F, bi, bj);
  const int e = blockIdx.y * blockDim.x + threadIdx.x;
  if (e >= GW_I * GW_J) return;
  const int64_t i = (int64_t)bi * GW_I + e / GW_J, j = (int64_t)bj * GW_J + e % GW_J;
  if (i > j || j >= F) return;
  int64_t acc[EX_SLOTS];
#pragma unroll
  for (int k = 0; k < EX_SLOTS; ++k) acc[k] = 0;
  const double* p = part + tile * (GW_I * GW_J) + e;
#pragma unroll 4
  for (int64_t sl = 0; sl < nslice; ++sl) ex_add(acc, p[sl * ntile * (GW_I * GW_J)]);
  const int64_t FF = F * F, o = i * F + j;
#pragma unroll
  for (int k = 0; k < EX_SLOTS; ++k) limbs[k * FF + o] = (accumulate ? limbs[k * FF + o] : 0) + acc[k];
  counts[o] = (accumulate ? counts[o] : 0) + (int64_t)ncnt[o];
}

}  // namespace fmx

struct DirectPlan {
  GramPlan g;                                   // g.ntile: k_gram_f64w tiles (256 x 128)
  int64_t nd, nwd, nw;
  int64_t zc_slices = 0, apad = 0;              // z-pass mode: slices per Zc chunk, padded row
  int64_t bits_bytes() const { return SmallPlan::align256((int64_t)sizeof(uint32_t) * F * nw); }
  int64_t part_bytes() const { return SmallPlan::align256((int64_t)sizeof(double) * g.nslice * g.ntile * GW_I * GW_J); }
  int64_t cnt_bytes() const { return (int64_t)sizeof(unsigned long long) * F * F; }
  int64_t inv_bytes() const {
    return zc_slices ? SmallPlan::align256((int64_t)sizeof(double) * F * zc_slices * FMX_GRAM_DATE_BLOCK * apad)
                     : SmallPlan::align256((int64_t)sizeof(double) * 2 * F * D);
  }
  int64_t bytes() const { return bits_bytes() + part_bytes() + SmallPlan::align256(cnt_bytes()) + inv_bytes(); }
  int64_t F, D;
};
// date slices for the direct Gram: enough workgroups for several rounds over the CUs and a
// count that fills the last round (136 upper tiles x 8 slices = 1088 workgroups left the
// fifth round of a one-workgroup-per-CU launch a quarter full)
static GramPlan direct_gram_plan(int64_t F, int64_t d0, int64_t d1, int slots) {
  GramPlan p;
  p.nb = 0;
  p.ntile = gw_ntile(F);
  const int64_t ndates = d1 - d0;
  const int64_t s0 = std::max<int64_t>(1, std::min<int64_t>(ndates, ceil_div((int64_t)4 * slots, p.ntile)));
  int64_t best = s0;
  double best_eff = 0.0;
  for (int64_t s = s0; s <= std::min<int64_t>(ndates, 4 * s0); ++s) {
    const int64_t wg = p.ntile * ceil_div(ndates, ceil_div(ndates, s));
    const double eff = (double)wg / (double)(ceil_div(wg, (int64_t)slots) * slots);
    if (eff > best_eff + 0.01) { best_eff = eff; best = s; }
  }
  p.dps = ceil_div(ndates, best);
  p.nslice = ceil_div(ndates, p.dps);
  return p;
}

static DirectPlan direct_plan(int64_t F, int64_t D, int64_t A, int64_t d0, int64_t d1) {
  DirectPlan p;
  p.F = F;
  p.D = D;
  (void)A;
  p.g = direct_gram_plan(F, d0, d1, 256);       // one k_gram_f64w workgroup per CU
  p.nd = d1 - d0;
  p.nwd = ceil_div(A, (int64_t)32);
  p.nw = p.nd * p.nwd;
  return p;
}

// N = M M^T of the validity bits [F][nw] into ncnt (zeroed by the caller): the i8-MFMA tile
// kernel, or (FMX_GRAM_CNT=0, the A/B arm) the AND / popcount kernel
static fmx_status launch_pair_counts(const uint32_t* bits, int64_t F, int64_t nw, unsigned long long* ncnt,
                                     hipStream_t st) {
  static const int mode = [] { const char* e = getenv("FMX_GRAM_CNT"); return e ? atoi(e) : 1; }();
  if (mode == 0) {
    const int T = (int)ceil_div(F, (int64_t)PF_T);
    const int ntp = T * (T + 1) / 2;
    // >= ~2048 workgroups: the word range is cut into pieces of whole 64-word chunks
    const int64_t nks = std::max<int64_t>(1, std::min<int64_t>(ceil_div(nw, (int64_t)4 * PF_W), 2048 / ntp + 1));
    const int64_t wps = ceil_div(ceil_div(nw, nks), (int64_t)PF_W) * PF_W;
    k_gram_popc_fm<<<dim3((unsigned)ntp, (unsigned)ceil_div(nw, wps)), 256, 0, st>>>(bits, F, nw, wps, ncnt);
    FMX_LAUNCH_CHECK("k_gram_popc_fm");
    return FMX_OK;
  }
  const int T = (int)ceil_div(F, (int64_t)GC_T);
  const int64_t ntp = (int64_t)T * (T + 1) / 2;
  // word slices: ~2 rounds of 4 workgroups per CU with a full last round, whole 16-word
  // chunks, and at most 2^25 words per slice (i32 accumulators: <= 32 bits per word)
  const int64_t nchunk = ceil_div(nw, (int64_t)GC_KW);
  int64_t nks = 1;
  double best = -1.0;
  for (int64_t k = 1; k <= std::min<int64_t>(nchunk, std::max<int64_t>(1, 4096 / ntp)); ++k) {
    const int64_t wg = ntp * k, slots = 1024;
    const double eff = (double)wg / (double)(ceil_div(wg, slots) * slots) - (wg < slots ? 1.0 : 0.0);
    if (eff > best + 0.01) { best = eff; nks = k; }
  }
  nks = std::max<int64_t>(nks, ceil_div(nw, (int64_t)1 << 25));
  const int64_t wps = ceil_div(ceil_div(nw, nks), (int64_t)GC_KW) * GC_KW;
  const dim3 grid((unsigned)ntp, (unsigned)ceil_div(nw, wps));
  if (nw % 4 == 0) k_gram_cnt_i8<true><<<grid, 256, 0, st>>>(bits, F, nw, wps, ncnt);
  else k_gram_cnt_i8<false><<<grid, 256, 0, st>>>(bits, F, nw, wps, ncnt);
  FMX_LAUNCH_CHECK("k_gram_cnt_i8");
  return FMX_OK;
}

// k_gram_db's counts: chunk-major bits [nw][F] into ncnt [FP][FP], every pair of the 16 x 16
// blocks on or above the block diagonal (FMX_GRAM_CNT=0: the AND / popcount kernel)
static fmx_status launch_pair_counts_cm(const uint32_t* mbits, int64_t F, int64_t nw, int FP,
                                        unsigned long long* ncnt, hipStream_t st) {
  static const int mode = [] { const char* e = getenv("FMX_GRAM_CNT"); return e ? atoi(e) : 1; }();
  if (mode == 0) {
    const int T = (int)ceil_div(F, (int64_t)32);
    const int ntile = T * (T + 1) / 2;
    const int64_t nks = std::max<int64_t>(1, std::min<int64_t>(ceil_div(nw, (int64_t)4 * PC_W), 2048 / ntile + 1));
    const int64_t wps = ceil_div(ceil_div(nw, nks), (int64_t)PC_W) * PC_W;
    const unsigned nky = (unsigned)ceil_div(nw, wps);
    k_gram_popc<<<dim3((unsigned)ntile, nky), 256, 0, st>>>(mbits, F, nw, wps, FP, ncnt);
    FMX_LAUNCH_CHECK("k_gram_popc");
    return FMX_OK;
  }
  const int T = (int)ceil_div(F, (int64_t)GC_T);
  const int64_t ntp = (int64_t)T * (T + 1) / 2;
  const int64_t nchunk = ceil_div(nw, (int64_t)GC_KW);
  // word slices: ~4 workgroups per CU, whole 16-word chunks, <= 2^25 words per slice
  int64_t nks = std::max<int64_t>(1, std::min<int64_t>(nchunk, 1024 / ntp));
  nks = std::max<int64_t>(nks, ceil_div(nw, (int64_t)1 << 25));
  const int64_t wps = ceil_div(ceil_div(nw, nks), (int64_t)GC_KW) * GC_KW;
  k_gram_cnt_i8<false, true><<<dim3((unsigned)ntp, (unsigned)ceil_div(nw, wps)), 256, 0, st>>>(mbits, F, nw, wps, ncnt,
                                                                                               (int64_t)FP, 1);
  FMX_LAUNCH_CHECK("k_gram_cnt_i8<cm>");
  return FMX_OK;
}

extern "C" int64_t fmx_gram_direct_work_bytes(int64_t F, int64_t D, int64_t A, int64_t d0, int64_t d1) {
  if (F <= 0 || d1 <= d0) return 0;
  return direct_plan(F, D, A, d0, d1).bytes();
}

extern "C" fmx_status fmx_gram_direct(const double* X, const double* stats, double* G, double* N, int64_t F,
                                      int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t d1, int32_t accumulate,
                                      void* work, int64_t work_bytes, void* stream) {
  FMX_ARG(X && stats && G && N, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && d0 >= 0 && d1 <= D && d0 <= d1, "bad dims");
  FMX_ARG(F <= 65535 && d1 - d0 <= 0x7fffffff, "too many factors / dates");
  if (F == 0 || d1 == d0) return FMX_OK;
  const DirectPlan pl = direct_plan(F, D, A, d0, d1);
  if (fmx_status e = check_work(work, work_bytes, pl.bytes(), "fmx_gram_direct_work_bytes")) return e;
  hipStream_t st = as_stream(stream);
  char* w = static_cast<char*>(work);
  const double* zst = stats;
  uint32_t* bits = reinterpret_cast<uint32_t*>(w);
  double* part = reinterpret_cast<double*>(w + pl.bits_bytes());
  unsigned long long* ncnt = reinterpret_cast<unsigned long long*>(w + pl.bits_bytes() + pl.part_bytes());
  double* zinv = reinterpret_cast<double*>(w + pl.bits_bytes() + pl.part_bytes() + SmallPlan::align256(pl.cnt_bytes()));
  // the tile kernel writes the validity bits (its diagonal tiles); an odd chunk count per
  // date leaves each date's last half-word unwritten: zero the bits first then
  if (ceil_div(A, (int64_t)GW_K) % 2 == 1) FMX_HIP(hipMemsetAsync(bits, 0, pl.bits_bytes(), st));
  k_inv_stats<<<(unsigned)ceil_div(F * D, (int64_t)256), 256, 0, st>>>(stats, zinv, F * D);
  FMX_LAUNCH_CHECK("k_inv_stats");
  zst = zinv;
  const void* k = (ld % 2 == 0) ? (const void*)k_gram_f64w<true> : (const void*)k_gram_f64w<false>;
  const size_t lds = GRAM_W_LDS;
  FMX_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int64_t dps = pl.g.dps, ntile = pl.g.ntile, nslice = pl.g.nslice;
  static const int xcd = [] { const char* e = getenv("FMX_GRAM_XCD"); return e ? atoi(e) : 1; }();
  int xcd_arg = xcd;
  const int64_t nwg = xcd == 1 ? 8 * ((ntile * nslice + 7) / 8) : ntile * nslice;
  uint16_t* bits16 = reinterpret_cast<uint16_t*>(bits);
  int64_t nwd = pl.nwd;
  static const int wopt = [] { const char* e = getenv("FMX_GRAM_WOPT"); return e ? atoi(e) : 1; }();
  int wopt_arg = wopt;
  int64_t phase = 0;
  void* args[] = {(void*)&X, (void*)&zst, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&d0, (void*)&d1,
                  (void*)&dps, (void*)&phase, (void*)&ntile, (void*)&nslice, (void*)&xcd_arg, (void*)&wopt_arg,
                  (void*)&part, (void*)&bits16, (void*)&nwd};
  const dim3 grid = xcd == 2 ? dim3((unsigned)ntile, (unsigned)nslice) : dim3((unsigned)nwg);
  FMX_HIP(hipLaunchKernel(k, grid, dim3(1024), args, lds, st));
  k_gram_reduce_w<<<dim3((unsigned)pl.g.ntile, GW_I * GW_J / 256), 256, 0, st>>>(part, pl.g.nslice, pl.g.ntile, F,
                                                                                 G, accumulate);
  FMX_LAUNCH_CHECK("k_gram_reduce_w");
  FMX_HIP(hipMemsetAsync(ncnt, 0, pl.cnt_bytes(), st));
  if (fmx_status e = launch_pair_counts(bits, F, pl.nw, ncnt, st)) return e;
  k_gram_counts<<<(unsigned)ceil_div(F * F, (int64_t)256), 256, 0, st>>>(ncnt, F, N, accumulate);
  FMX_LAUNCH_CHECK("k_gram_counts");
  return FMX_OK;
}

// Exact (GPU-count-independent) direct Gram: the tile kernel's date slices are ABSOLUTE
// blocks of FMX_GRAM_DATE_BLOCK dates (local row 0 = absolute date d_origin), each block's
// fp64 partial tiles fold into fixed-point limbs (exactsum.hpp).  A date shard whose bounds
// are multiples of the block holds whole blocks, so every block's partial -- and the integer
// sum over blocks and ranks -- is the same at 1, 2, 4 or 8 GPUs.
// z-pass mode (default where the row fits the register-resident moment kernel, A <= 8192;
// FMX_GRAM_ZC=0 keeps the stats + z-while-staging form): the dates run in chunks of
// zc_slices date blocks -- a z pass (row moments, Zc, validity bits) then the tile kernel on
// Zc with no staging arithmetic.  32 blocks of C4's 72 tiles make 9 full rounds of the CUs;
// the Zc chunk is capped at 32 GB (FMX_GRAM_ZC_GB).
static bool gram_zc_enabled(int64_t A) {
  static const int on = [] { const char* e = getenv("FMX_GRAM_ZC"); return e ? atoi(e) : 1; }();
  return on && gram_zc_fits(A);
}
static DirectPlan direct_exact_plan(int64_t F, int64_t D, int64_t A, int64_t d0, int64_t d1, int64_t phase,
                                    bool zc = false) {
  DirectPlan p;
  p.F = F;
  p.D = D;
  p.g.nb = 0;
  p.g.ntile = gw_ntile(F);
  p.g.dps = FMX_GRAM_DATE_BLOCK;
  p.g.nslice = ceil_div(d1 - d0 + phase, (int64_t)FMX_GRAM_DATE_BLOCK);
  p.nd = d1 - d0;
  p.nwd = ceil_div(A, (int64_t)32);
  p.nw = p.nd * p.nwd;
  if (zc) {
    p.apad = ceil_div(A, (int64_t)GW_K) * GW_K;
    const int64_t per_slice = (int64_t)sizeof(double) * F * FMX_GRAM_DATE_BLOCK * p.apad;
    // FMX_GRAM_ZC_GB (read per call): a smaller cap for runs that hold several shards'
    // workspaces on one device at once (the in-process 8-shard test); the blocks' exact
    // partials do not depend on the chunking
    const char* cap_e = getenv("FMX_GRAM_ZC_GB");
    const int64_t cap_gb = cap_e && atoi(cap_e) > 0 ? atoi(cap_e) : 32;
    p.zc_slices = std::max<int64_t>(1, std::min<int64_t>({(int64_t)32, p.g.nslice, (cap_gb << 30) / per_slice}));
  }
  return p;
}

static int64_t block_phase(int64_t d_origin, int64_t d0) {
  const int64_t a = d_origin + d0;
  return ((a % FMX_GRAM_DATE_BLOCK) + FMX_GRAM_DATE_BLOCK) % FMX_GRAM_DATE_BLOCK;
}

extern "C" int64_t fmx_gram_direct_exact_work_bytes(int64_t F, int64_t D, int64_t A, int64_t d0, int64_t d1,
                                                    int64_t d_origin) {
  if (F <= 0 || d1 <= d0) return 0;
  return direct_exact_plan(F, D, A, d0, d1, block_phase(d_origin, d0), gram_zc_enabled(A)).bytes();
}

extern "C" fmx_status fmx_gram_direct_exact(const double* X, const double* stats, int64_t* limbs, int64_t* counts,
                                            int64_t F, int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t d1,
                                            int64_t d_origin, int32_t accumulate, void* work, int64_t work_bytes,
                                            void* stream) {
  const bool zc = gram_zc_enabled(A);
  FMX_ARG(X && limbs && counts, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && d0 >= 0 && d1 <= D && d0 <= d1 && d_origin >= 0, "bad dims");
  FMX_ARG(F <= 65535 && d1 - d0 <= 0x7fffffff && A <= 0x7fffffff, "too many factors / dates / assets");
  hipStream_t st = as_stream(stream);
  if (!accumulate && F > 0) {
    FMX_HIP(hipMemsetAsync(limbs, 0, sizeof(int64_t) * FMX_GRAM_EXACT_SLOTS * F * F, st));
    FMX_HIP(hipMemsetAsync(counts, 0, sizeof(int64_t) * F * F, st));
  }
  if (F == 0 || d1 == d0 || A == 0) return FMX_OK;
  const int64_t phase = block_phase(d_origin, d0);
  const DirectPlan pl = direct_exact_plan(F, D, A, d0, d1, phase, zc);
  if (fmx_status e = check_work(work, work_bytes, pl.bytes(), "fmx_gram_direct_exact_work_bytes")) return e;
  char* w = static_cast<char*>(work);
  uint32_t* bits = reinterpret_cast<uint32_t*>(w);
  double* part = reinterpret_cast<double*>(w + pl.bits_bytes());
  unsigned long long* ncnt = reinterpret_cast<unsigned long long*>(w + pl.bits_bytes() + pl.part_bytes());
  double* zinv = reinterpret_cast<double*>(w + pl.bits_bytes() + pl.part_bytes() + SmallPlan::align256(pl.cnt_bytes()));
  if (zc) {
    // chunks of zc_slices absolute date blocks: z pass over the chunk's dates into Zc (the
    // zinv region), then the tile kernel on Zc; slice s of the whole range covers dates
    // [d0 + 16 s - phase, d0 + 16 (s + 1) - phase) clipped to [d0, d1)
    double* Zc = zinv;
    const int64_t ntile = pl.g.ntile, nsl = pl.g.nslice, dps = FMX_GRAM_DATE_BLOCK, apad = pl.apad, nwd = pl.nwd;
    // FMX_GRAM_GLDS: 0 register-staged k_gram_f64w<true, true>, 8 / 16 (default) waves of k_gram_zw
    static const int glds = [] { const char* e = getenv("FMX_GRAM_GLDS"); return e ? atoi(e) : 16; }();
    const void* k = glds == 8 ? (const void*)k_gram_zw<8> : glds ? (const void*)k_gram_zw<16>
                                                                 : (const void*)k_gram_f64w<true, true>;
    const int nthr = glds == 8 ? 512 : 1024;
    const size_t klds = glds ? GRAM_Z_LDS : GRAM_W_LDS;
    FMX_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)klds));
    for (int64_t s0 = 0; s0 < nsl; s0 += pl.zc_slices) {
      const int64_t s1 = std::min(nsl, s0 + pl.zc_slices);
      const int64_t dc0 = s0 == 0 ? d0 : d0 + s0 * dps - phase, dc1 = std::min(d1, d0 + s1 * dps - phase);
      const int64_t ndc = dc1 - dc0;
      if (fmx_status e = gram_zc_pass(X, F, D, A, ld, dc0, ndc, Zc, apad, bits + (dc0 - d0) * nwd, d1 - d0, nwd, st))
        return e;
      const double* zx = Zc;
      const double* znull = nullptr;
      int64_t Dz = ndc, Az = apad, lz = apad, z0 = 0, z1 = ndc, ph = s0 == 0 ? phase : 0, nsc = s1 - s0;
      int xcd_arg = 1, wopt_arg = 1;
      double* pc = part + s0 * ntile * (GW_I * GW_J);
      uint16_t* nob = nullptr;
      const int64_t nwg = 8 * ((ntile * nsc + 7) / 8);
      void* args[] = {(void*)&zx, (void*)&znull, (void*)&F, (void*)&Dz, (void*)&Az, (void*)&lz, (void*)&z0, (void*)&z1,
                      (void*)&dps, (void*)&ph, (void*)&ntile, (void*)&nsc, (void*)&xcd_arg, (void*)&wopt_arg,
                      (void*)&pc, (void*)&nob, (void*)&nwd};
      void* zargs[] = {(void*)&zx, (void*)&F, (void*)&Dz, (void*)&Az, (void*)&dps, (void*)&ph, (void*)&ntile, (void*)&nsc,
                       (void*)&pc};
      FMX_HIP(hipLaunchKernel(k, dim3((unsigned)nwg), dim3(nthr), glds ? zargs : args, klds, st));
    }
    FMX_HIP(hipMemsetAsync(ncnt, 0, pl.cnt_bytes(), st));
    if (fmx_status e = launch_pair_counts(bits, F, pl.nw, ncnt, st)) return e;
    k_gram_fold_w<<<dim3((unsigned)ntile, GW_I * GW_J / 256), 256, 0, st>>>(part, nsl, ntile, F, ncnt, limbs, counts,
                                                                            accumulate ? 1 : 0);
    FMX_LAUNCH_CHECK("k_gram_fold_w");
    return FMX_OK;
  }
  if (ceil_div(A, (int64_t)GW_K) % 2 == 1) FMX_HIP(hipMemsetAsync(bits, 0, pl.bits_bytes(), st));
  if (!stats) {                                   // no caller stats: the row moments in place
    if (fmx_status e = fmx_cs_moment_stats(FMX_CS_STATS, X, nullptr, F, D, A, ld, nullptr, zinv, stream)) return e;
    stats = zinv;
  }
  k_inv_stats<<<(unsigned)ceil_div(F * D, (int64_t)256), 256, 0, st>>>(stats, zinv, F * D);
  FMX_LAUNCH_CHECK("k_inv_stats");
  const double* zst = zinv;
  const void* k = (ld % 2 == 0) ? (const void*)k_gram_f64w<true> : (const void*)k_gram_f64w<false>;
  FMX_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)GRAM_W_LDS));
  int64_t dps = pl.g.dps, ntile = pl.g.ntile, nslice = pl.g.nslice, ph = phase, nwd = pl.nwd;
  int xcd_arg = 1, wopt_arg = 1;
  const int64_t nwg = 8 * ((ntile * nslice + 7) / 8);
  uint16_t* bits16 = reinterpret_cast<uint16_t*>(bits);
  void* args[] = {(void*)&X, (void*)&zst, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&d0, (void*)&d1,
                  (void*)&dps, (void*)&ph, (void*)&ntile, (void*)&nslice, (void*)&xcd_arg, (void*)&wopt_arg,
                  (void*)&part, (void*)&bits16, (void*)&nwd};
  FMX_HIP(hipLaunchKernel(k, dim3((unsigned)nwg), dim3(1024), args, GRAM_W_LDS, st));
  FMX_HIP(hipMemsetAsync(ncnt, 0, pl.cnt_bytes(), st));
  if (fmx_status e = launch_pair_counts(bits, F, pl.nw, ncnt, st)) return e;
  k_gram_fold_w<<<dim3((unsigned)ntile, GW_I * GW_J / 256), 256, 0, st>>>(part, nslice, ntile, F, ncnt, limbs, counts,
                                                                          accumulate ? 1 : 0);
  FMX_LAUNCH_CHECK("k_gram_fold_w");
  return FMX_OK;
}

extern "C" fmx_status fmx_greedy_prune(const double* C, int64_t F, int64_t ldc, const int64_t* order, int64_t n_order,
                                       double rho, int64_t top_x, int32_t* kept, int32_t* n_kept, void* stream) {
  FMX_ARG(C && order && kept && n_kept, "null pointer");
  FMX_ARG(F >= 0 && ldc >= F && n_order >= 0 && top_x >= 0, "bad dims");
  FMX_ARG((int64_t)sizeof(double) * F <= 160 * 1024, "too many factors for the LDS walk (F <= 20480)");
  hipStream_t st = as_stream(stream);
  const size_t lds = sizeof(double) * std::max<int64_t>(F, 1);
  if (lds > 64 * 1024)
    FMX_HIP(hipFuncSetAttribute((const void*)k_greedy_prune, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  k_greedy_prune<<<1, GP_NT, lds, st>>>(C, F, ldc, order, n_order, rho, top_x, kept, n_kept);
  FMX_LAUNCH_CHECK("k_greedy_prune");
  return FMX_OK;
}

extern "C" int64_t fmx_corr_prune_windows_work_bytes(int64_t F, int64_t D, int64_t J, int32_t window,
                                                     const int32_t* s0_host) {
  if (F <= 0 || J <= 0 || !s0_host) return 0;
  int64_t d_lo, nd;
  prune_dates(D, J, window, s0_host, d_lo, nd);
  return prune_part_bytes(F, nd) + (int64_t)sizeof(int32_t) * J;
}

extern "C" fmx_status fmx_corr_prune_windows(const double* X, const double* stats, int64_t F, int64_t D, int64_t A,
                                             int64_t ld, int64_t J, int32_t window, const int32_t* s0_host,
                                             const int32_t* order, const double* metrics, int32_t use_rank_icir,
                                             double threshold, double rho, int32_t top_x, double* w_out,
                                             void* work, int64_t work_bytes, void* stream) {
  FMX_ARG(X && stats && s0_host && order && metrics && w_out, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && J >= 0 && window >= 1 && top_x >= 0, "bad dims");
  if (F > 256) {
    set_error("fmx_corr_prune_windows keeps per-date F x F partials: F <= 256");
    return FMX_ERR_UNSUPPORTED;
  }
  if (F == 0 || J == 0) return FMX_OK;
  FMX_ARG(J <= 0x7fffffffll, "too many windows");
  if (fmx_status e = check_work(work, work_bytes, fmx_corr_prune_windows_work_bytes(F, D, J, window, s0_host),
                                "fmx_corr_prune_windows_work_bytes"))
    return e;
  hipStream_t st = as_stream(stream);
  char* w = static_cast<char*>(work);
  const int col = use_rank_icir ? 3 : 1;
  const int nb = (int)ceil_div(F, 16);
  switch (nb) {
#define FMX_WP(K)                                                                                            \
  case K:                                                                                                    \
    return window_prune_launch<K>(X, stats, F, D, A, ld, J, window, s0_host, order, metrics, col, threshold, \
                                  rho, top_x, w_out, w, st);
    FMX_WP(1) FMX_WP(2) FMX_WP(3) FMX_WP(4) FMX_WP(5) FMX_WP(6) FMX_WP(7) FMX_WP(8)
    FMX_WP(9) FMX_WP(10) FMX_WP(11) FMX_WP(12) FMX_WP(13) FMX_WP(14) FMX_WP(15) FMX_WP(16)
#undef FMX_WP
    default: return FMX_ERR_UNSUPPORTED;
  }
}
