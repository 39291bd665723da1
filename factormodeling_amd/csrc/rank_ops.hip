// Bucket-rank kernels (bucketrank.hpp): cs_rank (average/min/max), cs_winsor /
// cs_filter_center quantiles, and the fused multi-lag daily IC.
//
// Reference: operations.py:54-75 (cs_rank, cs_winsor, cs_filter_center) and
// factor_selector.py:36-48 (per-date pearsonr, pearsonr(rankdata), beta).
#include "bucketrank.hpp"

namespace fmx {

constexpr int BR_NT = 256;

template <int EMAX>
struct RowRegs {
  uint64_t key[EMAX];
  int bkt[EMAX];
};

// ------------------------------------------------------------------------------------
template <int EMAX>
__global__ void __launch_bounds__(BR_NT)
k_cs_rank_br(const double* __restrict__ X, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld, int method,
             const uint8_t* __restrict__ present) {
  __shared__ BRShared<BR_NT> S;
  extern __shared__ uint64_t bkey[];
  uint16_t* binfo = (uint16_t*)(bkey + A);
  uint16_t* bidx = binfo + A;
  const int t = threadIdx.x;
  const int64_t d = blockIdx.x, f = blockIdx.y;
  const double* x = X + (f * D + d) * ld;
  double* y = Y + (f * D + d) * ld;
  const uint8_t* prow = present ? present + d * ld : nullptr;
  RowRegs<EMAX> R;
  int nrow_l = 0, nv_l = 0;
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t i = t + (int64_t)k * BR_NT;
    R.key[k] = KEY_SENTINEL;
    if (i < A) {
      const bool p = prow ? prow[i] != 0 : true;
      const double v = x[i];
      nrow_l += p;
      if (p && v == v) { R.key[k] = okey(v); nv_l += 1; }
    }
  }
  int nrow, nv;
  block_exscan<BR_NT>(nrow_l, S.iscr, &nrow);
  block_exscan<BR_NT>(nv_l, S.iscr, &nv);
  if (method == FMX_RANK_AVERAGE_PROPAGATE && nv < nrow) {
    for (int64_t i = t; i < A; i += BR_NT) y[i] = qnan();
    return;
  }
  const bool half = (method != FMX_RANK_AVERAGE_PROPAGATE) && nrow == 1;
  {
    const int64_t pos = ((int64_t)t * A) / BR_NT;
    uint64_t sk = KEY_SENTINEL;
    if (pos < A && (prow ? prow[pos] != 0 : true)) {
      const double v = x[pos];
      if (v == v) sk = okey(v);
    }
    br_splitters<BR_NT>(S, sk);
  }
  for (int b = t; b < BRShared<BR_NT>::NB; b += BR_NT) { S.cnt[0][b] = 0; S.cursor[b] = 0; }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    R.bkt[k] = -1;
    if (R.key[k] != KEY_SENTINEL) {
      R.bkt[k] = bucket_of<BR_NT>(S, R.key[k]);
      atomicAdd(&S.cnt[0][R.bkt[k]], 1);
    }
  }
  __syncthreads();
  br_scan<BR_NT>(S, 1);
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t i = t + (int64_t)k * BR_NT;
    if (R.bkt[k] >= 0) {
      const int slot = S.start[0][R.bkt[k]] + atomicAdd(&S.cursor[R.bkt[k]], 1);
      bkey[slot] = R.key[k];
      binfo[slot] = (uint16_t)(R.bkt[k] | (1 << BR_MSHIFT));
      bidx[slot] = (uint16_t)i;
    } else if (i < A) {
      const bool p = prow ? prow[i] != 0 : true;
      y[i] = (p && half) ? 0.5 : qnan();
    }
  }
  __syncthreads();
  const double den = (double)(nrow - 1);
  for (int q = t; q < nv; q += BR_NT) {            // bucket order
    const uint64_t key = bkey[q];
    const int b = binfo[q] & ((1 << BR_MSHIFT) - 1);
    int lt, eq;
    br_inbucket<BR_NT>(S, bkey, binfo, b, key, 1, &lt, &eq);
    const int less = S.start[0][b] + lt;
    double r;
    if (method == FMX_RANK_MIN) r = (double)(less + 1);
    else if (method == FMX_RANK_MAX) r = (double)(less + eq);
    else r = (double)less + (double)(eq + 1) / 2.0;
    y[bidx[q]] = half ? 0.5 : (r - 1.0) / den;
  }
}

// ------------------------------------------------------------------------------------
// OP 0 = cs_winsor (clip to the quantiles when >= 5 non-NaN), 1 = cs_filter_center.
template <int OP, int EMAX>
__global__ void __launch_bounds__(BR_NT)
k_cs_quantile_br(const double* __restrict__ X, double* __restrict__ Y, int64_t D, int64_t A, int64_t ld,
                 double qlo, double qhi, const uint8_t* __restrict__ present) {
  __shared__ BRShared<BR_NT> S;
  __shared__ uint64_t bc;
  extern __shared__ uint64_t bkey[];
  const int t = threadIdx.x;
  const int64_t d = blockIdx.x, f = blockIdx.y;
  const double* x = X + (f * D + d) * ld;
  double* y = Y + (f * D + d) * ld;
  const uint8_t* prow = present ? present + d * ld : nullptr;
  RowRegs<EMAX> R;
  int nv_l = 0;
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t i = t + (int64_t)k * BR_NT;
    R.key[k] = KEY_SENTINEL;
    if (i < A && (prow ? prow[i] != 0 : true)) {
      const double v = x[i];
      if (v == v) { R.key[k] = okey(v); nv_l += 1; }
    }
  }
  int nv;
  block_exscan<BR_NT>(nv_l, S.iscr, &nv);
  double lo = qnan(), hi = qnan();
  if (nv > 0 && (OP == 1 || nv >= 5)) {
    const int64_t pos = ((int64_t)t * A) / BR_NT;
    uint64_t sk = KEY_SENTINEL;
    if (pos < A && (prow ? prow[pos] != 0 : true)) {
      const double v = x[pos];
      if (v == v) sk = okey(v);
    }
    br_splitters<BR_NT>(S, sk);
    for (int b = t; b < BRShared<BR_NT>::NB; b += BR_NT) { S.cnt[0][b] = 0; S.cursor[b] = 0; }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      R.bkt[k] = -1;
      if (R.key[k] != KEY_SENTINEL) {
        R.bkt[k] = bucket_of<BR_NT>(S, R.key[k]);
        atomicAdd(&S.cnt[0][R.bkt[k]], 1);
      }
    }
    __syncthreads();
    br_scan<BR_NT>(S, 1);
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (R.bkt[k] >= 0) {
        const int slot = S.start[0][R.bkt[k]] + atomicAdd(&S.cursor[R.bkt[k]], 1);
        bkey[slot] = R.key[k];
      }
    }
    __syncthreads();
    double qv[2];
    const double qs[2] = {qlo, qhi};
    for (int z = 0; z < 2; ++z) {
      // numpy linear percentile from order statistics p and p+1
      const double vi = (double)(nv - 1) * qs[z];
      double a, b, g;
      if (vi >= (double)(nv - 1)) {
        a = b = okey_inv(br_select<BR_NT, EMAX>(S, bkey, nv - 1, &bc));
        g = vi + 1.0;
      } else {
        const double pf = floor(vi);
        const int p = (int)pf;
        g = vi - pf;
        a = okey_inv(br_select<BR_NT, EMAX>(S, bkey, p, &bc));
        b = okey_inv(br_select<BR_NT, EMAX>(S, bkey, p + 1, &bc));
      }
      const double diff = b - a;
      qv[z] = (g >= 0.5) ? b - diff * (1.0 - g) : a + diff * g;
    }
    lo = qv[0];
    hi = qv[1];
  }
  for (int64_t i = t; i < A; i += BR_NT) {
    if (prow && !prow[i]) { y[i] = qnan(); continue; }
    const double v = x[i];
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
// stats of the pairs (X[f][s], R[s + L_m]) for up to two lags.  Mask bit 0 = non-NaN
// exposure (bucket layout), bit m (1..NL) = pair-valid for lag m.
template <int EMAX>
__global__ void __launch_bounds__(BR_NT)
k_ic_daily_br(const double* __restrict__ X, const double* __restrict__ Rt, int64_t F, int64_t D, int64_t A,
              int64_t ld, int L0, int L1, int NL, double* __restrict__ out) {
  __shared__ BRShared<BR_NT> S;
  extern __shared__ uint64_t bkey[];
  uint16_t* binfo = (uint16_t*)(bkey + A);
  uint16_t* bidx = binfo + A;
  const int t = threadIdx.x;
  const int64_t s = blockIdx.x, f = blockIdx.y;
  const double* xf = X + (f * D + s) * ld;
  const int lagv[2] = {L0, L1};
  const double* rr[2];
  bool act[2];
  for (int m = 0; m < 2; ++m) {
    act[m] = m < NL && s + lagv[m] < D;
    rr[m] = act[m] ? Rt + (s + lagv[m]) * ld : nullptr;
  }
  if (!act[0] && !act[1]) return;
  RowRegs<EMAX> R;
  uint8_t mem[EMAX];
  int nl[3] = {0, 0, 0};
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t i = t + (int64_t)k * BR_NT;
    R.key[k] = KEY_SENTINEL;
    mem[k] = 0;
    if (i < A) {
      const double v = xf[i];
      if (v == v) {
        R.key[k] = okey(v);
        uint8_t mm = 1;
        for (int m = 0; m < 2; ++m)
          if (act[m]) { const double r = rr[m][i]; if (r == r) mm |= (uint8_t)(2 << m); }
        mem[k] = mm;
        for (int m = 0; m < 3; ++m) nl[m] += (mm >> m) & 1;
      }
    }
  }
  int n[3];
  for (int m = 0; m < 3; ++m) block_exscan<BR_NT>(nl[m], S.iscr, &n[m]);
  const bool need = (act[0] && n[1] >= 3) || (act[1] && n[2] >= 3);
  if (need) {
    const int64_t pos = ((int64_t)t * A) / BR_NT;
    uint64_t sk = KEY_SENTINEL;
    if (pos < A) { const double v = xf[pos]; if (v == v) sk = okey(v); }
    br_splitters<BR_NT>(S, sk);
    for (int b = t; b < BRShared<BR_NT>::NB; b += BR_NT) {
      S.cnt[0][b] = S.cnt[1][b] = S.cnt[2][b] = 0;
      S.cursor[b] = 0;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      R.bkt[k] = -1;
      if (mem[k]) {
        const int b = bucket_of<BR_NT>(S, R.key[k]);
        R.bkt[k] = b;
        for (int m = 0; m < 3; ++m)
          if ((mem[k] >> m) & 1) atomicAdd(&S.cnt[m][b], 1);
      }
    }
    __syncthreads();
    br_scan<BR_NT>(S, 3);
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      if (R.bkt[k] >= 0) {
        const int slot = S.start[0][R.bkt[k]] + atomicAdd(&S.cursor[R.bkt[k]], 1);
        bkey[slot] = R.key[k];
        binfo[slot] = (uint16_t)(R.bkt[k] | ((int)mem[k] << BR_MSHIFT));
        bidx[slot] = (uint16_t)(t + k * BR_NT);
      }
    }
    __syncthreads();
  }
  // pass 1: means and constant checks per lag
  double v1[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // sf, sr per lag, then (-min f, max f) unused
  double fmn[2] = {INFINITY, INFINITY}, fmx[2] = {-INFINITY, -INFINITY};
  double rmn[2] = {INFINITY, INFINITY}, rmx[2] = {-INFINITY, -INFINITY};
#pragma unroll
  for (int k = 0; k < EMAX; ++k) {
    const int64_t i = t + (int64_t)k * BR_NT;
    if (!mem[k]) continue;
    const double fv = okey_inv(R.key[k]);
    for (int m = 0; m < 2; ++m) {
      if (!((mem[k] >> (m + 1)) & 1)) continue;
      const double r = rr[m][i];
      v1[2 * m] += fv;
      v1[2 * m + 1] += r;
      fmn[m] = fmin(fmn[m], fv); fmx[m] = fmax(fmx[m], fv);
      rmn[m] = fmin(rmn[m], r); rmx[m] = fmax(rmx[m], r);
    }
  }
  block_sum_vec<BR_NT, 4>(v1, S.dscr);
  double mm8[8] = {-fmn[0], fmx[0], -rmn[0], rmx[0], -fmn[1], fmx[1], -rmn[1], rmx[1]};
  for (int q = 0; q < 8; ++q)
    for (int o = 32; o > 0; o >>= 1) mm8[q] = fmax(mm8[q], __shfl_xor(mm8[q], o));
  {
    const int lane = t & 63, wid = t >> 6;
    if (lane == 0) for (int q = 0; q < 8; ++q) S.dscr[wid * 8 + q] = mm8[q];
    __syncthreads();
    for (int q = 0; q < 8; ++q) {
      double z = -INFINITY;
      for (int w = 0; w < BR_NT / 64; ++w) z = fmax(z, S.dscr[w * 8 + q]);
      mm8[q] = z;
    }
    __syncthreads();
  }
  double fm[2], rm[2], km[2];
  for (int m = 0; m < 2; ++m) {
    const double dn = (double)n[m + 1];
    fm[m] = v1[2 * m] / dn;
    rm[m] = v1[2 * m + 1] / dn;
    km[m] = (dn + 1.0) / 2.0;
  }
  // pass 2: centred moments with in-group ranks
  double v2[14];
  for (int q = 0; q < 14; ++q) v2[q] = 0.0;
  if (need) {
    for (int q = t; q < n[0]; q += BR_NT) {         // bucket order
      const uint64_t key = bkey[q];
      const int info = binfo[q];
      const int mm = info >> BR_MSHIFT;
      if (!(mm & 6)) continue;
      const int64_t i = bidx[q];
      const int b = info & ((1 << BR_MSHIFT) - 1);
      int lt[3], eq[3];
      br_inbucket<BR_NT>(S, bkey, binfo, b, key, 3, lt, eq);
      const double fv = okey_inv(key);
      for (int m = 0; m < 2; ++m) {
        if (!((mm >> (m + 1)) & 1)) continue;
        const int less = S.start[m + 1][b] + lt[m + 1];
        const double rk = (double)less + (double)(eq[m + 1] + 1) / 2.0;
        const double r = rr[m][i];
        const double dx = fv - fm[m], dy = r - rm[m], dk = rk - km[m];
        double* w = v2 + 7 * m;
        w[0] += dx * dy; w[1] += dx * dx; w[2] += dy * dy;
        w[3] += dk * dy; w[4] += dk * dk;
        w[5] += fv * fv; w[6] += fv * r;
      }
    }
  }
  block_sum_vec<BR_NT, 14>(v2, S.dscr);
  if (t == 0) {
    for (int m = 0; m < 2; ++m) {
      if (!act[m]) continue;
      const int64_t td = s + lagv[m];
      double* o = out + ((int64_t)(m * 4) * F + f) * D + td;
      const int64_t st = F * D;
      const int nn = n[m + 1];
      double ic = qnan(), ric = qnan(), beta = qnan();
      if (nn >= 3) {
        const double* w = v2 + 7 * m;
        const bool fconst = (-mm8[4 * m + 0]) == mm8[4 * m + 1];
        const bool rconst = (-mm8[4 * m + 2]) == mm8[4 * m + 3];
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
}

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

template <class K>
static fmx_status launch_br(K kern_table, int64_t A, dim3 grid, void** args, hipStream_t st) {
  const int E = (int)ceil_div(std::max<int64_t>(A, 1), BR_NT);
  const void* k = kern_table(E);
  if (!k) { set_error("row too long for the bucket-rank kernels (A > 16384)"); return FMX_ERR_UNSUPPORTED; }
  const size_t lds = (size_t)A * 12 + 16;
  if (lds > 64 * 1024) FMX_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  FMX_HIP(hipLaunchKernel(k, grid, dim3(BR_NT), args, lds, st));
  return FMX_OK;
}

#define FMX_EMAX_TABLE(KT)                                                   \
  [](int E) -> const void* {                                                 \
    if (E <= 4) return (const void*)KT<4>;                                   \
    if (E <= 8) return (const void*)KT<8>;                                   \
    if (E <= 16) return (const void*)KT<16>;                                 \
    if (E <= 24) return (const void*)KT<24>;                                 \
    if (E <= 32) return (const void*)KT<32>;                                 \
    if (E <= 40) return (const void*)KT<40>;                                 \
    if (E <= 64) return (const void*)KT<64>;                                 \
    return (const void*)nullptr;                                             \
  }

template <int E> constexpr auto kq0 = k_cs_quantile_br<0, E>;
template <int E> constexpr auto kq1 = k_cs_quantile_br<1, E>;

}  // namespace fmx

using namespace fmx;

// Internal entry points used by cs_ops.hip / ic.hip dispatch.
namespace fmx {

fmx_status br_cs_rank(const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld, int method,
                      const uint8_t* present, hipStream_t st) {
  void* args[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&method, (void*)&present};
  return launch_br(FMX_EMAX_TABLE(k_cs_rank_br), A, dim3((unsigned)D, (unsigned)F), args, st);
}

fmx_status br_cs_quantile(int op, const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                          double qlo, double qhi, const uint8_t* present, hipStream_t st) {
  void* args[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&qlo, (void*)&qhi, (void*)&present};
  if (op == 0) return launch_br(FMX_EMAX_TABLE(kq0), A, dim3((unsigned)D, (unsigned)F), args, st);
  return launch_br(FMX_EMAX_TABLE(kq1), A, dim3((unsigned)D, (unsigned)F), args, st);
}

fmx_status br_ic_daily(const double* X, const double* R, int64_t F, int64_t D, int64_t A, int64_t ld,
                       const int32_t* lags_host, int n_lags, double* out, hipStream_t st) {
  for (int base = 0; base < n_lags; base += 2) {
    int NL = std::min(2, n_lags - base);
    int L0 = lags_host[base], L1 = NL > 1 ? lags_host[base + 1] : 0;
    double* o = out + (int64_t)base * 4 * F * D;
    k_ic_empty<<<(unsigned)F, 64, 0, st>>>(o, F, D, L0, L1, NL);
    FMX_LAUNCH_CHECK("k_ic_empty");
    void* args[] = {(void*)&X, (void*)&R, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&L0, (void*)&L1,
                    (void*)&NL, (void*)&o};
    fmx_status e = launch_br(FMX_EMAX_TABLE(k_ic_daily_br), A, dim3((unsigned)D, (unsigned)F), args, st);
    if (e) return e;
  }
  return FMX_OK;
}

}  // namespace fmx
