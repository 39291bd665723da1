// Composite factors (composite_factor.py:137-342).
//
// composite_factor_calculation (:137-218)
//   k_comp_adj      per (column, date): suffix preprocessing with numpy linear
//                   nanpercentiles of that column's values (:157-178)
//   k_comp_proxy    per (prefix group, date): skipna mean over the group's columns (:181-190)
//   (normalise)     fmx_cs_moment(MARKET_NEUTRALIZE) == safe_zcol (:195-204) or
//                   fmx_cs_rank with scipy NaN propagation (:206-210)
//   k_comp_combine  per date: skipna mean (zscore) / skipna sum (rank) over proxies, then
//                   demean with a numpy-exact pairwise mean (:216)
// weighted_composite_factor (:220-342): the same stages driven by a per-selection-date
// plan (selected columns, suffix pools, prefix groups, group weights) built on the host;
// percentiles are pooled over all selected columns that share a suffix (:251-268).
//
// Order statistics use a block radix select over order-preserving 64-bit keys read
// from global memory (8 passes of 8-bit digits), so pooled rows of any length work.
#include "rowkit.hpp"

namespace fmx {

constexpr int CP_NT = 256;

// k-th smallest (0-based) order-preserving key among the n values produced by val(i)
// (NaN skipped).  hist: LDS int[256]; scr: LDS uint64[4].
template <class Val>
__device__ uint64_t block_select_kth(Val val, int64_t n, int64_t k, int* hist, uint64_t* scr) {
  uint64_t prefix = 0, mask = 0;
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int b = threadIdx.x; b < 256; b += CP_NT) hist[b] = 0;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < n; i += CP_NT) {
      double v = val(i);
      if (v != v) continue;
      uint64_t key = okey(v);
      if ((key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t acc = 0;
      int b = 0;
      for (; b < 256; ++b) {
        if (acc + hist[b] > k) break;
        acc += hist[b];
      }
      scr[0] = (uint64_t)b;
      scr[1] = (uint64_t)(k - acc);
    }
    __syncthreads();
    const uint64_t b = scr[0];
    k = (int64_t)scr[1];
    prefix |= b << shift;
    mask |= (uint64_t)255 << shift;
    __syncthreads();
  }
  return prefix;
}

// numpy percentile(method='linear') at fraction q over the non-NaN values (count nv > 0).
template <class Val>
__device__ double block_percentile(Val val, int64_t n, int64_t nv, double q, int* hist, uint64_t* scr,
                                   double* dscr) {
  const double vi = (double)(nv - 1) * q;
  double a, b, g;
  if (vi >= (double)(nv - 1)) {
    uint64_t k = block_select_kth(val, n, nv - 1, hist, scr);
    a = b = okey_inv(k);
    g = vi + 1.0;
  } else {
    const double pf = floor(vi);
    const int64_t p = (int64_t)pf;
    g = vi - pf;
    uint64_t kp = block_select_kth(val, n, p, hist, scr);
    // (p+1)-th: kp itself if more than p+1 values are <= kp, else the smallest key > kp
    int cle = 0;
    uint64_t nxt = KEY_SENTINEL;
    for (int64_t i = threadIdx.x; i < n; i += CP_NT) {
      double v = val(i);
      if (v != v) continue;
      uint64_t key = okey(v);
      cle += key <= kp;
      if (key > kp && key < nxt) nxt = key;
    }
    // block reductions (sum of cle, min of nxt)
    for (int o = 32; o > 0; o >>= 1) {
      cle += __shfl_xor(cle, o);
      uint64_t t = __shfl_xor(nxt, o);
      nxt = t < nxt ? t : nxt;
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) hist[wid] = cle;
    __syncthreads();
    if (lane == 0) dscr[wid] = __longlong_as_double((long long)nxt);
    __syncthreads();
    int tc = 0;
    uint64_t tn = KEY_SENTINEL;
    for (int w = 0; w < CP_NT / 64; ++w) {
      tc += hist[w];
      uint64_t t = (uint64_t)__double_as_longlong(dscr[w]);
      tn = t < tn ? t : tn;
    }
    __syncthreads();
    a = okey_inv(kp);
    b = (tc > p + 1) ? a : okey_inv(tn);
  }
  const double diff = b - a;
  return (g >= 0.5) ? b - diff * (1.0 - g) : a + diff * g;
}

__device__ __forceinline__ double suffix_scale(int suf, double s, double lo, double hi) {
  if (suf == 1) return (s <= lo) ? -1.0 : ((s >= hi) ? 1.0 : 0.0);   // _eq (NaN -> 0)
  double c = s < lo ? lo : (s > hi ? hi : s);                          // np.clip keeps NaN
  if (suf == 2) return ((c - lo) / (hi - lo)) * 2.0 - 1.0;             // _flx
  if (suf == 3) return (c - lo) / (hi - lo);                           // _long
  return (c - hi) / (hi - lo);                                         // _short
}

// ---------------------------------------------------------------------------------------
// composite_factor_calculation: per (selected column j, date d)
__global__ void __launch_bounds__(CP_NT)
k_comp_adj(const double* __restrict__ X, const int32_t* __restrict__ cols, const int32_t* __restrict__ suffix,
           const double* __restrict__ qlo, const double* __restrict__ qhi, double* __restrict__ Adj, int64_t D,
           int64_t A) {
  __shared__ int hist[256];
  __shared__ uint64_t scr[4];
  __shared__ double dscr[8];
  const int64_t d = blockIdx.x, j = blockIdx.y;
  const double* x = X + ((int64_t)cols[j] * D + d) * A;
  double* o = Adj + (j * D + d) * A;
  const int suf = suffix[j];
  if (suf == 0) {
    for (int64_t a = threadIdx.x; a < A; a += CP_NT) o[a] = x[a];
    return;
  }
  int c = 0;
  for (int64_t a = threadIdx.x; a < A; a += CP_NT) c += x[a] == x[a];
  int nv;
  block_exscan<CP_NT>(c, hist, &nv);
  if (nv == 0) {
    for (int64_t a = threadIdx.x; a < A; a += CP_NT) o[a] = 0.0;
    return;
  }
  auto val = [&](int64_t i) { return x[i]; };
  const double lo = block_percentile(val, A, nv, qlo[suf], hist, scr, dscr);
  const double hi = block_percentile(val, A, nv, qhi[suf], hist, scr, dscr);
  for (int64_t a = threadIdx.x; a < A; a += CP_NT) o[a] = (hi == lo) ? 0.0 : suffix_scale(suf, x[a], lo, hi);
}

// skipna mean over the columns of each prefix group.  gcols: concatenated column lists,
// goff[g]..goff[g+1].  Sequential sum in column order (DataFrame.mean(axis=1)).
__global__ void k_comp_proxy(const double* __restrict__ Adj, const int32_t* __restrict__ gcols,
                             const int32_t* __restrict__ goff, double* __restrict__ Prox, int64_t D, int64_t A) {
  const int64_t d = blockIdx.x, g = blockIdx.y;
  for (int64_t a = threadIdx.x; a < A; a += blockDim.x) {
    double s = 0.0;
    int c = 0;
    for (int q = goff[g]; q < goff[g + 1]; ++q) {
      double v = Adj[((int64_t)gcols[q] * D + d) * A + a];
      if (v == v) { s += v; c += 1; }
    }
    Prox[(g * D + d) * A + a] = c ? s / (double)c : qnan();
  }
}

// per date: combine G normalised proxies (mode 0: skipna mean, 1: skipna sum), demean.
__global__ void __launch_bounds__(CP_NT)
k_comp_combine(const double* __restrict__ Nrm, int64_t G, int64_t D, int64_t A, int mode, PwTable pw,
               const uint8_t* __restrict__ present, double* __restrict__ Out) {
  extern __shared__ double row[];
  double* nodes = row + A;
  int* iscr = (int*)(nodes + (2 * (A / 64) + 8));
  const int64_t d = blockIdx.x;
  const uint8_t* prow = present ? present + d * A : nullptr;
  int cl = 0;
  for (int64_t a = threadIdx.x; a < A; a += CP_NT) {
    if (prow && !prow[a]) { row[a] = qnan(); continue; }
    double s = 0.0;
    int c = 0;
    for (int64_t g = 0; g < G; ++g) {
      double v = Nrm[(g * D + d) * A + a];
      if (v == v) { s += v; c += 1; }
    }
    double r = (mode == 0) ? (c ? s / (double)c : qnan()) : s;
    row[a] = r;
    cl += r == r;
  }
  int cnt;
  block_exscan<CP_NT>(cl, iscr, &cnt);
  const double sum = block_pw_sum<CP_NT>([&](int i) { double t = row[i]; return t == t ? t : 0.0; },
                                         pw.get((int)A), nodes);
  const double mean = cnt ? sum / (double)cnt : qnan();
  for (int64_t a = threadIdx.x; a < A; a += CP_NT) Out[d * A + a] = row[a] - mean;
}

// ---------------------------------------------------------------------------------------
// weighted_composite_factor.  Plan per selection row j (panel date pdate[j]):
//   ncol[j], col[j][k], suf[j][k], grp[j][k] (k < KMAX), ngrp[j], gw[j][g] (g < KMAX)
// pooled percentiles per (selection row j, suffix s): the columns of row j with suffix s
// are listed (in selection order) in scol[soff[j*4+s-1] .. soff[j*4+s]).
__global__ void __launch_bounds__(CP_NT)
k_wcomp_pct(const double* __restrict__ X, const int32_t* __restrict__ pdate, const int32_t* __restrict__ soff,
            const int32_t* __restrict__ scol, int64_t D, int64_t A, const double* __restrict__ qlo,
            const double* __restrict__ qhi, double* __restrict__ lohi) {
  __shared__ int hist[256];
  __shared__ uint64_t scr[4];
  __shared__ double dscr[8];
  const int64_t j = blockIdx.x;
  const int s = blockIdx.y + 1;  // suffix 1..4
  double* o = lohi + (j * 4 + (s - 1)) * 3;
  const int64_t d = pdate[j];
  const int c0 = soff[j * 4 + s - 1], m = soff[j * 4 + s] - c0;
  if (m == 0 || d < 0) {
    if (threadIdx.x == 0) { o[0] = o[1] = qnan(); o[2] = -1.0; }
    return;
  }
  const int32_t* cs = scol + c0;
  auto val = [&](int64_t i) { int64_t q = i / A; return X[((int64_t)cs[q] * D + d) * A + (i - q * A)]; };
  const int64_t n = (int64_t)m * A;
  int c = 0;
  for (int64_t i = threadIdx.x; i < n; i += CP_NT) { double v = val(i); c += v == v; }
  int nv;
  block_exscan<CP_NT>(c, hist, &nv);
  if (nv == 0) {
    if (threadIdx.x == 0) { o[0] = o[1] = qnan(); o[2] = 0.0; }
    return;
  }
  const double lo = block_percentile(val, n, nv, qlo[s], hist, scr, dscr);
  const double hi = block_percentile(val, n, nv, qhi[s], hist, scr, dscr);
  if (threadIdx.x == 0) { o[0] = lo; o[1] = hi; o[2] = (double)nv; }
}

__global__ void k_wcomp_proxy(const double* __restrict__ X, const int32_t* __restrict__ pdate,
                              const int32_t* __restrict__ ncol, const int32_t* __restrict__ col,
                              const int32_t* __restrict__ suf, const int32_t* __restrict__ grp, int KMAX, int64_t D,
                              int64_t A, const double* __restrict__ lohi, int64_t J, double* __restrict__ Prox) {
  const int64_t j = blockIdx.x, g = blockIdx.y;
  const int64_t d = pdate[j];
  double* o = Prox + (g * J + j) * A;
  const int nc = ncol[j];
  for (int64_t a = threadIdx.x; a < A; a += blockDim.x) {
    double s = 0.0;
    int c = 0;
    bool any = false;
    for (int k = 0; k < nc; ++k) {
      if (grp[j * KMAX + k] != g) continue;
      any = true;
      const int sf = suf[j * KMAX + k];
      double v = X[((int64_t)col[j * KMAX + k] * D + d) * A + a];
      if (sf > 0) {
        const double* lh = lohi + (j * 4 + (sf - 1)) * 3;
        if (lh[2] == 0.0 || lh[0] == lh[1]) v = 0.0;     // clean.size == 0 or lo == hi
        else v = suffix_scale(sf, v, lh[0], lh[1]);
      }
      if (v == v) { s += v; c += 1; }
    }
    o[a] = (any && c) ? s / (double)c : qnan();
  }
}

__global__ void __launch_bounds__(CP_NT)
k_wcomp_combine(const double* __restrict__ Nrm, const int32_t* __restrict__ pdate, const int32_t* __restrict__ ngrp,
                const double* __restrict__ gw, int KMAX, int64_t J, int64_t D, int64_t A, PwTable pw,
                const uint8_t* __restrict__ present, double* __restrict__ Out) {
  extern __shared__ double row[];
  double* nodes = row + A;
  int* iscr = (int*)(nodes + (2 * (A / 64) + 8));
  const int64_t j = blockIdx.x;
  const int64_t d = pdate[j];
  const int ng = ngrp[j];
  if (d < 0 || ng == 0) return;
  const uint8_t* prow = present ? present + d * A : nullptr;
  int cl = 0;
  for (int64_t a = threadIdx.x; a < A; a += CP_NT) {
    if (prow && !prow[a]) { row[a] = qnan(); continue; }
    double s = 0.0;                                   // Python sum(): 0 + n0*w0 + n1*w1 ...
    for (int g = 0; g < ng; ++g) s = s + Nrm[((int64_t)g * J + j) * A + a] * gw[j * KMAX + g];
    row[a] = s;
    cl += s == s;
  }
  int cnt;
  block_exscan<CP_NT>(cl, iscr, &cnt);
  const double sum = block_pw_sum<CP_NT>([&](int i) { double t = row[i]; return t == t ? t : 0.0; },
                                         pw.get((int)A), nodes);
  const double mean = cnt ? sum / (double)cnt : qnan();
  for (int64_t a = threadIdx.x; a < A; a += CP_NT) {
    double v = row[a] - mean;
    Out[d * A + a] = (v == v) ? v : 0.0;            // reindex(...).fillna(0)
  }
}

}  // namespace fmx

using namespace fmx;

extern "C" fmx_status fmx_comp_adj(const double* X, const int32_t* cols_dev, const int32_t* suffix_dev,
                                   const double* qlo_dev, const double* qhi_dev, double* Adj, int64_t K, int64_t D,
                                   int64_t A, void* stream) {
  FMX_ARG(X && cols_dev && suffix_dev && qlo_dev && qhi_dev && Adj, "null pointer");
  FMX_ARG(K >= 0 && D >= 0 && A >= 0, "bad dims");
  if (K == 0 || D == 0 || A == 0) return FMX_OK;
  k_comp_adj<<<dim3((unsigned)D, (unsigned)K), CP_NT, 0, as_stream(stream)>>>(X, cols_dev, suffix_dev, qlo_dev,
                                                                             qhi_dev, Adj, D, A);
  FMX_LAUNCH_CHECK("k_comp_adj");
  return FMX_OK;
}

extern "C" fmx_status fmx_comp_proxy(const double* Adj, const int32_t* gcols_dev, const int32_t* goff_dev,
                                     double* Prox, int64_t G, int64_t D, int64_t A, void* stream) {
  FMX_ARG(Adj && gcols_dev && goff_dev && Prox, "null pointer");
  if (G == 0 || D == 0 || A == 0) return FMX_OK;
  k_comp_proxy<<<dim3((unsigned)D, (unsigned)G), 256, 0, as_stream(stream)>>>(Adj, gcols_dev, goff_dev, Prox, D, A);
  FMX_LAUNCH_CHECK("k_comp_proxy");
  return FMX_OK;
}

static fmx_status combine_lds(const void* k, int64_t A, size_t* lds) {
  *lds = (size_t)A * 8 + (2 * (A / 64) + 8) * 8 + 16 * 4 + 64;
  if (*lds > 160 * 1024) { set_error("A too large for the combine kernel"); return FMX_ERR_UNSUPPORTED; }
  if (*lds > 64 * 1024) FMX_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)*lds));
  return FMX_OK;
}

extern "C" fmx_status fmx_comp_combine(const double* Nrm, int64_t G, int64_t D, int64_t A, int32_t mode,
                                       const uint8_t* present, double* Out, void* stream) {
  FMX_ARG(Nrm && Out, "null pointer");
  if (D == 0 || A == 0) return FMX_OK;
  fmx_status e = FMX_OK;
  PwTable pw = pw_table((int)A, &e);
  if (e) return e;
  size_t lds;
  if ((e = combine_lds((const void*)k_comp_combine, A, &lds))) return e;
  int m = mode;
  void* args[] = {(void*)&Nrm, (void*)&G, (void*)&D, (void*)&A, (void*)&m, (void*)&pw, (void*)&present, (void*)&Out};
  FMX_HIP(hipLaunchKernel((const void*)k_comp_combine, dim3((unsigned)D), dim3(CP_NT), args, lds, as_stream(stream)));
  return FMX_OK;
}

extern "C" fmx_status fmx_wcomp_pct(const double* X, const int32_t* pdate, const int32_t* soff, const int32_t* scol,
                                    int64_t J, int64_t D, int64_t A, const double* qlo_dev, const double* qhi_dev,
                                    double* lohi, void* stream) {
  FMX_ARG(X && pdate && soff && scol && qlo_dev && qhi_dev && lohi, "null pointer");
  if (J == 0) return FMX_OK;
  k_wcomp_pct<<<dim3((unsigned)J, 4), CP_NT, 0, as_stream(stream)>>>(X, pdate, soff, scol, D, A, qlo_dev, qhi_dev,
                                                                     lohi);
  FMX_LAUNCH_CHECK("k_wcomp_pct");
  return FMX_OK;
}

extern "C" fmx_status fmx_wcomp_proxy(const double* X, const int32_t* pdate, const int32_t* ncol, const int32_t* col,
                                      const int32_t* suf, const int32_t* grp, int32_t KMAX, int64_t J, int64_t D,
                                      int64_t A, const double* lohi, int64_t G, double* Prox, void* stream) {
  FMX_ARG(X && pdate && ncol && col && suf && grp && lohi && Prox, "null pointer");
  if (J == 0 || G == 0) return FMX_OK;
  k_wcomp_proxy<<<dim3((unsigned)J, (unsigned)G), 256, 0, as_stream(stream)>>>(X, pdate, ncol, col, suf, grp, KMAX, D,
                                                                              A, lohi, J, Prox);
  FMX_LAUNCH_CHECK("k_wcomp_proxy");
  return FMX_OK;
}

extern "C" fmx_status fmx_wcomp_combine(const double* Nrm, const int32_t* pdate, const int32_t* ngrp,
                                        const double* gw, int32_t KMAX, int64_t J, int64_t D, int64_t A,
                                        const uint8_t* present, double* Out, void* stream) {
  FMX_ARG(Nrm && pdate && ngrp && gw && Out, "null pointer");
  if (J == 0 || A == 0) return FMX_OK;
  fmx_status e = FMX_OK;
  PwTable pw = pw_table((int)A, &e);
  if (e) return e;
  size_t lds;
  if ((e = combine_lds((const void*)k_wcomp_combine, A, &lds))) return e;
  int km = KMAX;
  void* args[] = {(void*)&Nrm, (void*)&pdate, (void*)&ngrp, (void*)&gw, (void*)&km, (void*)&J, (void*)&D, (void*)&A,
                  (void*)&pw, (void*)&present, (void*)&Out};
  FMX_HIP(hipLaunchKernel((const void*)k_wcomp_combine, dim3((unsigned)J), dim3(CP_NT), args, lds, as_stream(stream)));
  return FMX_OK;
}
