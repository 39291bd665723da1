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
  const int nt = br_nt(1024);
  // counters, then keys [A] + member info [A] + lag masks [A] (k_ic_daily_fr)
  const size_t lds_fr = std::max<size_t>((size_t)(FRG<FR_K_IC>::NB + 1) * 8, (size_t)A * 13 + 16);
  auto fr_table = FMX_EMAX_TABLE(k_ic_daily_fr);
  const bool fine = rank_impl() == RANK_IMPL_FINE && lds_fits(fr_table(nt, br_emax(A, nt)), lds_fr);
  const size_t lds = fine ? lds_fr : (size_t)std::max<int64_t>(A, nt) * 8 + (size_t)((A + 15) & ~15ll);
  for (int base = 0; base < n_lags; base += 2) {
    int NL = std::min(2, n_lags - base);
    int L0 = lags_host[base], L1 = NL > 1 ? lags_host[base + 1] : 0;
    double* o = out + (int64_t)base * 4 * F * D;
    k_ic_empty<<<(unsigned)F, 64, 0, st>>>(o, F, D, L0, L1, NL);
    FMX_LAUNCH_CHECK("k_ic_empty");
    void* args[] = {(void*)&X, (void*)&R, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&L0, (void*)&L1,
                    (void*)&NL, (void*)&o};
    fmx_status e = fine ? launch_br(fr_table, nt, A, F * D, lds, args, st)
                        : launch_br(FMX_EMAX_TABLE(k_ic_daily_br), nt, A, F * D, lds, args, st);
    if (e) return e;
  }
  return FMX_OK;
}

// Daily IC from the doubled ranks of the same panel (k_ic_ranked): A <= 16384.
fmx_status br_ic_ranked(const double* X, const uint32_t* RK, const double* R, int64_t F, int64_t D, int64_t A,
                        int64_t ld, const int32_t* lags_host, int n_lags, double* out, hipStream_t st) {
  const int nt = 1024;
  if (br_emax(A, nt) < 0) { set_error("row too long for the ranked IC kernel (A > 16384)"); return FMX_ERR_UNSUPPORTED; }
  for (int base = 0; base < n_lags; base += 2) {
    int NL = std::min(2, n_lags - base);
    int L0 = lags_host[base], L1 = NL > 1 ? lags_host[base + 1] : 0;
    double* o = out + (int64_t)base * 4 * F * D;
    k_ic_empty<<<(unsigned)F, 64, 0, st>>>(o, F, D, L0, L1, NL);
    FMX_LAUNCH_CHECK("k_ic_empty");
    void* args[] = {(void*)&X, (void*)&RK, (void*)&R, (void*)&F, (void*)&D, (void*)&A, (void*)&ld, (void*)&L0,
                    (void*)&L1, (void*)&NL, (void*)&o};
    fmx_status e = launch_br(FMX_EMAX_TABLE(k_ic_ranked), nt, A, F * D, 0, args, st);
    if (e) return e;
  }
  return FMX_OK;
}

}  // namespace fmx

BR_PHASE_EXPORT(fmx_debug_phase_ic)
