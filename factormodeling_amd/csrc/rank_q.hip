// cs_winsor / cs_filter_center launcher (rank_kernels.hpp).
// Reference: operations.py:64-75
#include "rank_fine.hpp"
#include "rank_launch.hpp"

namespace fmx {

template <int NT, int E> constexpr auto kq0 = k_cs_quantile_br<0, NT, E>;
template <int NT, int E> constexpr auto kq1 = k_cs_quantile_br<1, NT, E>;

template <int NT, int E> constexpr auto kqf0 = k_cs_quantile_fa<0, NT, E, false>;
template <int NT, int E> constexpr auto kqf1 = k_cs_quantile_fa<1, NT, E, false>;
template <int NT, int E> constexpr auto kqf0p = k_cs_quantile_fa<0, NT, E, true>;
template <int NT, int E> constexpr auto kqf1p = k_cs_quantile_fa<1, NT, E, true>;

fmx_status br_cs_quantile(int op, const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                          double qlo, double qhi, const uint8_t* present, hipStream_t st) {
  void* args[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&qlo, (void*)&qhi, (void*)&present};
  // fine-bucket order statistics (default) or the splitter-bucket kernel (FMX_RANK_IMPL=br)
  if (rank_impl() == RANK_IMPL_FINE) {
    const int ntf = 512;
    const size_t lds_f = (size_t)FR_CS_WORDS * 4;
    const int E = br_emax(A, ntf);
    const void* k = op == 0 ? (present ? FMX_EMAX_TABLE(kqf0p)(ntf, E) : FMX_EMAX_TABLE(kqf0)(ntf, E))
                            : (present ? FMX_EMAX_TABLE(kqf1p)(ntf, E) : FMX_EMAX_TABLE(kqf1)(ntf, E));
    if (k && lds_fits(k, lds_f)) {
      if (F * D > 0x7fffffffll) { set_error("too many rows for one launch"); return FMX_ERR_UNSUPPORTED; }
      if (F * D == 0) return FMX_OK;
      FMX_HIP(hipLaunchKernel(k, fmx_grid2(D, F), dim3(ntf), args, lds_f, st));
      return FMX_OK;
    }
  }
  const int nt = br_nt(512);
  const size_t lds = (size_t)4 * QCAP * 8;
  if (op == 0) return launch_br(FMX_EMAX_TABLE(kq0), nt, A, D, F, lds, args, st);
  return launch_br(FMX_EMAX_TABLE(kq1), nt, A, D, F, lds, args, st);
}

}  // namespace fmx

BR_PHASE_EXPORT(fmx_debug_phase_q)
