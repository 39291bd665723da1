// cs_rank(method='first' | 'dense') for rows longer than the LDS bitonic kernel takes
// (operations.py:54-62: pandas Series.rank(method) over the date's non-NaN rows, then
// (r - 1) / (len - 1) with len counting the NaN rows; a single-row date -> 0.5).
//
// 'first' and 'dense' need the full order of each row (ties broken by position, or the
// count of distinct values below), which the fine-bucket kernels do not materialise.  A
// row of 16384 keys + indices does not fit one workgroup's LDS, so the rows are sorted in
// HBM instead: keys = order-preserving u64 of the value (sentinel for NaN / absent rows),
// values = the asset index; rocPRIM's segmented radix sort (stable: equal keys keep
// ascending asset order = pandas 'first') sorts a chunk of rows, then one workgroup per
// row walks its sorted run and scatters the ranks.  Chunks of rows bound the workspace.
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

// one workgroup per sorted row: counts, NaN / absent outputs, then the ranks
__global__ void __launch_bounds__(RS_NT)
k_rs_rank(const uint64_t* __restrict__ keys, const uint16_t* __restrict__ idx, const double* __restrict__ X,
          const uint8_t* __restrict__ present, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld, int64_t row0,
          int method) {
  __shared__ int iscr[RS_NT / 64 + 1];
  const int64_t r = blockIdx.x, row = row0 + r;
  const uint64_t* k = keys + r * A;
  const uint16_t* ix = idx + r * A;
  const double* x = X + row * ld;
  double* y = Y + row * ld;
  const uint8_t* prow = present ? present + (row % D) * ld : nullptr;
  int nrow_l = 0, nv_l = 0;
  for (int64_t a = threadIdx.x; a < A; a += RS_NT) {
    const bool p = prow ? prow[a] != 0 : true;
    nrow_l += p;
    nv_l += k[a] != KEY_SENTINEL;                 // sorted run: valid keys first
  }
  int nrow, nv;
  block_exscan<RS_NT>(nrow_l, iscr, &nrow);
  block_exscan<RS_NT>(nv_l, iscr, &nv);
  const bool half = nrow == 1;
  for (int64_t a = threadIdx.x; a < A; a += RS_NT) {
    const bool p = prow ? prow[a] != 0 : true;
    if (!p) y[a] = qnan();
    else if (!(x[a] == x[a])) y[a] = half ? 0.5 : qnan();
  }
  const double den = (double)(nrow - 1);
  // each thread walks a contiguous run of sorted positions; 'dense' needs the number of
  // value changes before the run (block exclusive scan of the per-run counts)
  const int C = (nv + RS_NT - 1) / RS_NT;
  const int p0 = min(nv, (int)threadIdx.x * C), p1 = min(nv, p0 + C);
  int base = 0;
  if (method == FMX_RANK_DENSE) {
    int c = 0;
    for (int p = p0; p < p1; ++p) c += (p == 0 || k[p] != k[p - 1]);
    int tot;
    base = block_exscan<RS_NT>(c, iscr, &tot);
  }
  for (int p = p0; p < p1; ++p) {
    double rk;
    if (method == FMX_RANK_DENSE) {
      base += (p == 0 || k[p] != k[p - 1]);
      rk = (double)base;
    } else {
      rk = (double)(p + 1);
    }
    y[ix[p]] = half ? 0.5 : (rk - 1.0) / den;
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

static int64_t al256(int64_t b) { return (b + 255) / 256 * 256; }

}  // namespace fmx

using namespace fmx;

extern "C" int64_t fmx_cs_rank_sorted_work_bytes(int64_t F, int64_t D, int64_t A) {
  if (F <= 0 || D <= 0 || A <= 0) return 0;
  const int64_t cr = rs_chunk_rows(F * D, A), n = cr * A;
  return 2 * al256(n * 8) + 2 * al256(n * 2) + al256((int64_t)rs_temp_bytes(cr, A));
}

extern "C" fmx_status fmx_cs_rank_sorted(const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                                         int32_t method, const uint8_t* present, void* work, int64_t work_bytes,
                                         void* stream) {
  FMX_ARG(X && Y, "null panel");
  FMX_ARG(F >= 0 && D >= 0 && A >= 0 && ld >= A && A <= 65535, "bad dims");
  FMX_ARG(method == FMX_RANK_FIRST || method == FMX_RANK_DENSE, "fmx_cs_rank_sorted: methods first / dense");
  if (F == 0 || D == 0 || A == 0) return FMX_OK;
  const int64_t need = fmx_cs_rank_sorted_work_bytes(F, D, A);
  if (!work || work_bytes < need) {
    set_error("workspace smaller than fmx_cs_rank_sorted_work_bytes()");
    return FMX_ERR_ARG;
  }
  hipStream_t st = as_stream(stream);
  const int64_t rows = F * D, cr = rs_chunk_rows(rows, A), n = cr * A;
  char* w = static_cast<char*>(work);
  uint64_t* kin = reinterpret_cast<uint64_t*>(w);
  uint64_t* kout = reinterpret_cast<uint64_t*>(w + al256(n * 8));
  uint16_t* vin = reinterpret_cast<uint16_t*>(w + 2 * al256(n * 8));
  uint16_t* vout = reinterpret_cast<uint16_t*>(w + 2 * al256(n * 8) + al256(n * 2));
  void* tmp = w + 2 * al256(n * 8) + 2 * al256(n * 2);
  const size_t tcap = (size_t)(need - (2 * al256(n * 8) + 2 * al256(n * 2)));
  for (int64_t r0 = 0; r0 < rows; r0 += cr) {
    const int64_t nr = std::min(cr, rows - r0);
    k_rs_keys<<<dim3((unsigned)ceil_div(A, RS_NT), (unsigned)nr), RS_NT, 0, st>>>(X, present, D, A, ld, r0, kin, vin);
    FMX_LAUNCH_CHECK("k_rs_keys");
    size_t tb = tcap;
    RowIter off(rocprim::counting_iterator<unsigned>(0), RowStart{(unsigned)A});
    FMX_HIP(rocprim::segmented_radix_sort_pairs(tmp, tb, kin, kout, vin, vout, (unsigned)(nr * A), (unsigned)nr, off,
                                                off + 1, 0, 64, st));
    k_rs_rank<<<(unsigned)nr, RS_NT, 0, st>>>(kout, vout, X, present, Y, D, A, ld, r0, method);
    FMX_LAUNCH_CHECK("k_rs_rank");
  }
  return FMX_OK;
}
