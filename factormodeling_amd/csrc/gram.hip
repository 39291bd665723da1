// Factor x factor correlation GEMM (builder-defined).
//
// C = (sum_d Z_d^T Z_d) / (sum_d M_d^T M_d) where Z are per-date z-scored exposures
// (NaN -> 0) and M the validity masks.  The reduction dimension K = dates x assets is
// huge (12.6e6 at 2520 x 5000) while F is 200..2000, so the Gram is computed as 64x64
// output tiles (upper triangle only) x K-slices (date ranges), each a workgroup of 4
// waves doing 2x2 v_mfma_f64_16x16x4_f64 tiles, with the K-slices reduced in a fixed
// order by a second kernel (deterministic; identical for any slice->XCD placement).
#include <algorithm>
#include <vector>

#include "rowkit.hpp"

namespace fmx {

typedef double dbl4 __attribute__((ext_vector_type(4)));

constexpr int GT = 64;    // output tile
constexpr int GK = 32;    // K step staged in LDS
constexpr int GKP = GK + 2;  // padded LDS row (conflict-free ds_read_b64)

// per-date z-score of one (f, d) row; builder spec: mean/std(ddof=0) over non-NaN,
// NaN -> 0, sigma in {0, NaN} -> whole row 0 and M = 0.
__global__ void __launch_bounds__(256)
k_zscore_exposures(const double* __restrict__ X, double* __restrict__ Z, double* __restrict__ M, int64_t D,
                   int64_t A, int64_t ld) {
  __shared__ double dscr[16];
  const int64_t d = blockIdx.x, f = blockIdx.y;
  const double* x = X + (f * D + d) * ld;
  double* z = Z + (f * D + d) * ld;
  double* m = M + (f * D + d) * ld;
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
    m[a] = valid ? 1.0 : 0.0;
  }
}

// Partial Gram of one upper-triangular 64x64 tile over dates [ds, de).
__global__ void __launch_bounds__(256)
k_gram_partial(const double* __restrict__ Z, int64_t F, int64_t D, int64_t A, int64_t ld, int64_t d0,
               int64_t d1, int64_t dates_per_slice, const int32_t* __restrict__ tile_i,
               const int32_t* __restrict__ tile_j, int64_t ntile, double* __restrict__ part) {
  __shared__ double As[GT * GKP];
  __shared__ double Bs[GT * GKP];
  const int64_t tile = blockIdx.x, slice = blockIdx.y;
  const int i0 = tile_i[tile] * GT, j0 = tile_j[tile] * GT;
  const int64_t ds = d0 + slice * dates_per_slice;
  const int64_t de = min<int64_t>(d1, ds + dates_per_slice);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  dbl4 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[m][n] = dbl4{0.0, 0.0, 0.0, 0.0};
  // loader mapping: 256 threads x 8 doubles = 64 rows x 32 k
  const int lr = tid >> 2, lc = (tid & 3) * 8;
  const bool rowA = (i0 + lr) < F, rowB = (j0 + lr) < F;
  for (int64_t d = ds; d < de; ++d) {
    const double* za = Z + ((int64_t)(i0 + lr) * D + d) * ld;
    const double* zb = Z + ((int64_t)(j0 + lr) * D + d) * ld;
    for (int64_t a0 = 0; a0 < A; a0 += GK) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        int64_t a = a0 + lc + u;
        As[lr * GKP + lc + u] = (rowA && a < A) ? za[a] : 0.0;
        Bs[lr * GKP + lc + u] = (rowB && a < A) ? zb[a] : 0.0;
      }
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < GK; kk += 4) {
        const int k = kk + (lane >> 4);
        double af[2], bf[2];
#pragma unroll
        for (int m = 0; m < 2; ++m) af[m] = As[(wr * 32 + m * 16 + (lane & 15)) * GKP + k];
#pragma unroll
        for (int n = 0; n < 2; ++n) bf[n] = Bs[(wc * 32 + n * 16 + (lane & 15)) * GKP + k];
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[m], bf[n], acc[m][n], 0, 0, 0);
      }
      __syncthreads();
    }
  }
  // C/D layout (f64 16x16x4): col = lane & 15, row = (lane >> 4) + 4 * reg
  double* p = part + (slice * ntile + tile) * (GT * GT);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int row = wr * 32 + m * 16 + (lane >> 4) + 4 * r;
        int col = wc * 32 + n * 16 + (lane & 15);
        p[row * GT + col] = acc[m][n][r];
      }
}

// Sum the slices in order and scatter the tile (and its mirror) into G[F][F].
__global__ void k_gram_reduce(const double* __restrict__ part, int64_t nslice, int64_t ntile,
                              const int32_t* __restrict__ tile_i, const int32_t* __restrict__ tile_j, int64_t F,
                              double* __restrict__ G, int accumulate) {
  const int64_t tile = blockIdx.x;
  const int i0 = tile_i[tile] * GT, j0 = tile_j[tile] * GT;
  for (int e = threadIdx.x; e < GT * GT; e += blockDim.x) {
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

extern "C" fmx_status fmx_zscore_exposures(const double* X, double* Z, double* M, int64_t F, int64_t D, int64_t A,
                                           int64_t ld, void* stream) {
  FMX_ARG(X && Z && M, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A, "bad dims");
  if (F == 0 || D == 0) return FMX_OK;
  k_zscore_exposures<<<dim3((unsigned)D, (unsigned)F), 256, 0, as_stream(stream)>>>(X, Z, M, D, A, ld);
  FMX_LAUNCH_CHECK("k_zscore_exposures");
  return FMX_OK;
}

static fmx_status gram_one(const double* Z, double* G, int64_t F, int64_t D, int64_t A, int64_t ld, int64_t d0,
                           int64_t d1, int accumulate, hipStream_t st) {
  const int nb = (int)ceil_div(F, GT);
  std::vector<int32_t> ti, tj;
  for (int i = 0; i < nb; ++i)
    for (int j = i; j < nb; ++j) { ti.push_back(i); tj.push_back(j); }
  const int64_t ntile = (int64_t)ti.size();
  const int64_t ndates = d1 - d0;
  // enough slices to fill the chip (>= ~1024 workgroups), at least one date each
  int64_t nslice = std::max<int64_t>(1, std::min<int64_t>(ndates, ceil_div(2048, ntile)));
  const int64_t dps = ceil_div(ndates, nslice);
  nslice = ceil_div(ndates, dps);
  int32_t* tdev = nullptr;
  double* part = nullptr;
  FMX_HIP(hipMallocAsync((void**)&tdev, sizeof(int32_t) * 2 * ntile, st));
  FMX_HIP(hipMallocAsync((void**)&part, sizeof(double) * nslice * ntile * GT * GT, st));
  std::vector<int32_t> packed(ti);
  packed.insert(packed.end(), tj.begin(), tj.end());
  FMX_HIP(hipMemcpyAsync(tdev, packed.data(), sizeof(int32_t) * 2 * ntile, hipMemcpyHostToDevice, st));
  FMX_HIP(hipStreamSynchronize(st));  // packed is a host temporary
  k_gram_partial<<<dim3((unsigned)ntile, (unsigned)nslice), 256, 0, st>>>(Z, F, D, A, ld, d0, d1, dps, tdev,
                                                                            tdev + ntile, ntile, part);
  FMX_LAUNCH_CHECK("k_gram_partial");
  k_gram_reduce<<<(unsigned)ntile, 256, 0, st>>>(part, nslice, ntile, tdev, tdev + ntile, F, G, accumulate);
  FMX_LAUNCH_CHECK("k_gram_reduce");
  FMX_HIP(hipFreeAsync(part, st));
  FMX_HIP(hipFreeAsync(tdev, st));
  return FMX_OK;
}

extern "C" fmx_status fmx_gram(const double* Z, const double* M, double* G, double* N, int64_t F, int64_t D,
                               int64_t A, int64_t ld, int64_t d0, int64_t d1, int32_t accumulate, void* stream) {
  FMX_ARG(Z && G, "null pointer");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && d0 >= 0 && d1 <= D && d0 <= d1, "bad dims");
  if (F == 0 || d1 == d0) return FMX_OK;
  hipStream_t st = as_stream(stream);
  fmx_status e = gram_one(Z, G, F, D, A, ld, d0, d1, accumulate, st);
  if (e || !M || !N) return e;
  return gram_one(M, N, F, D, A, ld, d0, d1, accumulate, st);
}
