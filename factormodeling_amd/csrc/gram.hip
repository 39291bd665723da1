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
#include <vector>

#include "rowkit.hpp"

namespace fmx {

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef float flt16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef double dbl2 __attribute__((ext_vector_type(2)));

constexpr int GT = 128;        // output tile
constexpr int GK = 32;         // fp64 K chunk staged in LDS
constexpr int GKP = GK + 2;    // padded row: bank = (4 r + 2 k) mod 64, conflict-free ds_read_b64
constexpr int MK = 64;         // bf16 K chunk
constexpr int MKP = MK + 8;    // padded row (16 B)

// per-date z-score of one (f, d) row; builder spec: mean/std(ddof=0) over non-NaN,
// NaN -> 0, sigma in {0, NaN} -> whole row 0 and M = 0.  M is written as bf16 0/1.
__global__ void __launch_bounds__(256)
k_zscore_exposures(const double* __restrict__ X, double* __restrict__ Z, uint16_t* __restrict__ M, int64_t D,
                   int64_t A, int64_t ld) {
  __shared__ double dscr[16];
  const int64_t d = blockIdx.x, f = blockIdx.y;
  const double* x = X + (f * D + d) * ld;
  double* z = Z + (f * D + d) * ld;
  uint16_t* m = M + (f * D + d) * ld;
  double s = 0.0, c = 0.0;
  for (int64_t a = threadIdx.x; a < A; a += 256) {
    double v = x[a];
    if (v == v) { s += v; c += 1.0; }
  }
  s = block_sum<256>(s, dscr);
  c = block_sum<256>(c, dscr);
  const double mean = c > 0 ? s / c : qnan();
  double q = 0.0;
  for (int64_t a = threadIdx.x; a < A; a += 256) {
    double v = x[a];
    if (v == v) q += (v - mean) * (v - mean);
  }
  q = block_sum<256>(q, dscr);
  const double sd = c > 0 ? sqrt(q / c) : qnan();
  const bool ok = sd > 0.0;
  for (int64_t a = threadIdx.x; a < ld; a += 256) {
    double v = a < A ? x[a] : qnan();
    bool valid = ok && v == v;
    z[a] = valid ? (v - mean) / sd : 0.0;
    m[a] = valid ? (uint16_t)0x3f80 : (uint16_t)0;   // bf16 1.0 / 0.0
  }
}

// ---------------------------------------------------------------------------------------
template <bool VEC>
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
      r[u] = (rowok && a < A) ? row[a] : 0.0;
    }
  }
}

template <bool VEC>
__global__ void __launch_bounds__(512)
k_gram_f64(const double* __restrict__ Z, int64_t F, int64_t D, int64_t A, int64_t ld, int64_t d0, int64_t d1,
           int64_t dates_per_slice, const int32_t* __restrict__ tile_i, const int32_t* __restrict__ tile_j,
           int64_t ntile, double* __restrict__ part) {
  __shared__ double As[GT * GKP];
  __shared__ double Bs[GT * GKP];
  const int64_t tile = blockIdx.x, slice = blockIdx.y;
  const int i0 = tile_i[tile] * GT, j0 = tile_j[tile] * GT;
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
  if (total > 0) issue(0);
  for (int64_t c = 0; c < total; ++c) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      As[lr * GKP + lc + u] = ra[u];
      Bs[lr * GKP + lc + u] = rb[u];
    }
    __syncthreads();
    if (c + 1 < total) issue(c + 1);   // next chunk in flight during the MFMAs
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
    __syncthreads();
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
            int64_t dates_per_slice, const int32_t* __restrict__ tile_i, const int32_t* __restrict__ tile_j,
            int64_t ntile, double* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) uint16_t As[GT * MKP];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[GT * MKP];
  const int64_t tile = blockIdx.x, slice = blockIdx.y;
  const int i0 = tile_i[tile] * GT, j0 = tile_j[tile] * GT;
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
  for (int64_t d = ds; d < de; ++d) {
    const uint16_t* ma = M + ((int64_t)(i0 + lr) * D + d) * ld;
    const uint16_t* mb = M + ((int64_t)(j0 + lr) * D + d) * ld;
    for (int64_t a0 = 0; a0 < A; a0 += MK) {
      if (vec && a0 + lc + 32 <= A) {
        const bf16x8* pa = reinterpret_cast<const bf16x8*>(ma + a0 + lc);
        const bf16x8* pb = reinterpret_cast<const bf16x8*>(mb + a0 + lc);
        bf16x8 za = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          *reinterpret_cast<bf16x8*>(&As[lr * MKP + lc + 8 * u]) = rowA ? pa[u] : za;
          *reinterpret_cast<bf16x8*>(&Bs[lr * MKP + lc + 8 * u]) = rowB ? pb[u] : za;
        }
      } else {
#pragma unroll
        for (int u = 0; u < 32; ++u) {
          const int64_t a = a0 + lc + u;
          As[lr * MKP + lc + u] = (rowA && a < A) ? ma[a] : (uint16_t)0;
          Bs[lr * MKP + lc + u] = (rowB && a < A) ? mb[a] : (uint16_t)0;
        }
      }
      __syncthreads();
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
__global__ void k_gram_reduce(const double* __restrict__ part, int64_t nslice, int64_t ntile,
                              const int32_t* __restrict__ tile_i, const int32_t* __restrict__ tile_j, int64_t F,
                              double* __restrict__ G, int accumulate) {
  const int64_t tile = blockIdx.x;
  const int i0 = tile_i[tile] * GT, j0 = tile_j[tile] * GT;
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

}  // namespace fmx

using namespace fmx;

extern "C" fmx_status fmx_zscore_exposures(const double* X, double* Z, uint16_t* M, int64_t F, int64_t D, int64_t A,
                                           int64_t ld, void* stream) {
  FMX_ARG(X && Z && M, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A, "bad dims");
  if (F == 0 || D == 0) return FMX_OK;
  k_zscore_exposures<<<dim3((unsigned)D, (unsigned)F), 256, 0, as_stream(stream)>>>(X, Z, M, D, A, ld);
  FMX_LAUNCH_CHECK("k_zscore_exposures");
  return FMX_OK;
}

static fmx_status gram_run(const void* Zp, bool mask, double* G, int64_t F, int64_t D, int64_t A, int64_t ld,
                           int64_t d0, int64_t d1, int accumulate, hipStream_t st) {
  const int nb = (int)ceil_div(F, GT);
  std::vector<int32_t> packed;
  for (int i = 0; i < nb; ++i)
    for (int j = i; j < nb; ++j) packed.push_back(i);
  const int64_t ntile = (int64_t)packed.size();
  for (int i = 0; i < nb; ++i)
    for (int j = i; j < nb; ++j) packed.push_back(j);
  const int64_t ndates = d1 - d0;
  // >= ~1024 workgroups to fill 256 CUs; bf16 slices must stay < 2^24 (date, asset) pairs
  int64_t nslice = std::max<int64_t>(1, std::min<int64_t>(ndates, ceil_div(1024, ntile)));
  int64_t dps = ceil_div(ndates, nslice);
  if (mask) {
    const int64_t cap = std::max<int64_t>(1, ((int64_t)1 << 24) / std::max<int64_t>(A, 1) - 1);
    dps = std::min(dps, cap);
  }
  nslice = ceil_div(ndates, dps);
  int32_t* tdev = nullptr;
  double* part = nullptr;
  FMX_HIP(hipMallocAsync((void**)&tdev, sizeof(int32_t) * 2 * ntile, st));
  FMX_HIP(hipMallocAsync((void**)&part, sizeof(double) * nslice * ntile * GT * GT, st));
  FMX_HIP(hipMemcpyAsync(tdev, packed.data(), sizeof(int32_t) * 2 * ntile, hipMemcpyHostToDevice, st));
  FMX_HIP(hipStreamSynchronize(st));  // packed is a host temporary
  dim3 grid((unsigned)ntile, (unsigned)nslice);
  if (mask) {
    k_gram_mask<<<grid, 256, 0, st>>>((const uint16_t*)Zp, F, D, A, ld, d0, d1, dps, tdev, tdev + ntile, ntile, part);
    FMX_LAUNCH_CHECK("k_gram_mask");
  } else if (ld % 2 == 0) {
    k_gram_f64<true><<<grid, 512, 0, st>>>((const double*)Zp, F, D, A, ld, d0, d1, dps, tdev, tdev + ntile, ntile,
                                           part);
    FMX_LAUNCH_CHECK("k_gram_f64");
  } else {
    k_gram_f64<false><<<grid, 512, 0, st>>>((const double*)Zp, F, D, A, ld, d0, d1, dps, tdev, tdev + ntile, ntile,
                                            part);
    FMX_LAUNCH_CHECK("k_gram_f64");
  }
  k_gram_reduce<<<dim3((unsigned)ntile, GT * GT / 256), 256, 0, st>>>(part, nslice, ntile, tdev, tdev + ntile, F, G,
                                                                      accumulate);
  FMX_LAUNCH_CHECK("k_gram_reduce");
  FMX_HIP(hipFreeAsync(part, st));
  FMX_HIP(hipFreeAsync(tdev, st));
  return FMX_OK;
}

extern "C" fmx_status fmx_gram(const double* Z, const uint16_t* M, double* G, double* N, int64_t F, int64_t D,
                               int64_t A, int64_t ld, int64_t d0, int64_t d1, int32_t accumulate, void* stream) {
  FMX_ARG(Z && G, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && d0 >= 0 && d1 <= D && d0 <= d1, "bad dims");
  if (F == 0 || d1 == d0) return FMX_OK;
  hipStream_t st = as_stream(stream);
  fmx_status e = gram_run(Z, false, G, F, D, A, ld, d0, d1, accumulate, st);
  if (e || !M || !N) return e;
  return gram_run(M, true, N, F, D, A, ld, d0, d1, accumulate, st);
}
