// cs_winsor / cs_filter_center launcher (rank_kernels.hpp).
// Reference: operations.py:64-75
#include "rank_launch.hpp"

namespace fmx {

template <int NT, int E> constexpr auto kq0 = k_cs_quantile_br<0, NT, E>;
template <int NT, int E> constexpr auto kq1 = k_cs_quantile_br<1, NT, E>;

fmx_status br_cs_quantile(int op, const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld,
                          double qlo, double qhi, const uint8_t* present, hipStream_t st) {
  void* args[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&qlo, (void*)&qhi, (void*)&present};
  const int nt = br_nt(512);
  const size_t lds = (size_t)4 * QCAP * 8;
  if (op == 0) return launch_br(FMX_EMAX_TABLE(kq0), nt, A, F * D, lds, args, st);
  return launch_br(FMX_EMAX_TABLE(kq1), nt, A, F * D, lds, args, st);
}

}  // namespace fmx

BR_PHASE_EXPORT(fmx_debug_phase_q)
