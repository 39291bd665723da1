// cs_rank launcher: persistent fine-bucket kernels (rank_fine.hpp) by default, the
// splitter-bucket kernels (rank_kernels.hpp) with FMX_RANK_IMPL=br or when a row does not
// fit the fine kernel's LDS.
// Reference: operations.py:54-62
#include "rank_fine.hpp"
#include "rank_launch.hpp"

namespace fmx {

template <int NT, int E> constexpr auto kcr_dense = k_cs_rank_fa<NT, E, false>;
template <int NT, int E> constexpr auto kcr_pres = k_cs_rank_fa<NT, E, true>;
template <int NT, int E> constexpr auto kcrw_dense = k_cs_rank_fa<NT, E, false, true>;
template <int NT, int E> constexpr auto kcrw_pres = k_cs_rank_fa<NT, E, true, true>;

fmx_status br_cs_rank(const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld, int method,
                      const uint8_t* present, hipStream_t st) {
  const int nt = br_nt(1024);
  const int nt_fa = fa_nt(A) == 1024 ? 1024 : 512;
  const size_t lds_fr = std::max<size_t>((size_t)A * 8, (size_t)FR_CS_WORDS * 4);
  const void* kfr = present ? FMX_EMAX_TABLE(kcr_pres)(nt_fa, br_emax(A, nt_fa))
                            : FMX_EMAX_TABLE(kcr_dense)(nt_fa, br_emax(A, nt_fa));
  if (rank_impl() == RANK_IMPL_BR || !lds_fits(kfr, lds_fr)) {
    void* args[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&method, (void*)&present};
    const size_t lds = (size_t)std::max<int64_t>(A, nt) * 8;
    return launch_br(FMX_EMAX_TABLE(k_cs_rank_br), nt, A, D, F, lds, args, st);
  }
  double* Y2 = nullptr;
  double qlo = 0.0, qhi = 0.0;
  fmx_rank2_t* RK = nullptr;
  FrIc ic{};
  FrZn zn{};
  const FrListLds ll = fr_list_lds(kfr, A, (size_t)fr_list_off(A, FR_CS_WORDS), 0);
  int lcap = ll.cap;
  void* args[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&method, (void*)&present,
                  (void*)&Y2, (void*)&qlo, (void*)&qhi, (void*)&RK, (void*)&ic, (void*)&zn, (void*)&lcap};
  if (F * D > 0x7fffffffll) { set_error("too many rows for one launch"); return FMX_ERR_UNSUPPORTED; }
  if (F * D == 0) return FMX_OK;
  FMX_HIP(set_dyn_lds(kfr, ll.bytes));
  FMX_HIP(hipLaunchKernel(kfr, fmx_grid2(D, F), dim3(nt_fa), args, ll.bytes, st));
  return FMX_OK;
}

// cs_rank (method average) and cs_winsor of the same rows in one pass (k_cs_rank_fa<WQ>),
// optionally the doubled ranks RK; returns FMX_ERR_UNSUPPORTED when the row does not fit
// the fine kernel (caller splits).
fmx_status br_cs_rank_winsor(const double* X, double* Yr, double* Yw, int64_t F, int64_t D, int64_t A, int64_t ld,
                             double qlo, double qhi, const uint8_t* present, fmx_rank2_t* RK, hipStream_t st) {
  const int nt_fa = fa_nt(A) == 1024 ? 1024 : 512;
  const size_t lds_fr = std::max<size_t>((size_t)A * 8, (size_t)FR_CS_WORDS * 4);
  const int E = br_emax(A, nt_fa);
  const void* k = present ? FMX_EMAX_TABLE(kcrw_pres)(nt_fa, E) : FMX_EMAX_TABLE(kcrw_dense)(nt_fa, E);
  if (rank_impl() == RANK_IMPL_BR || E < 0 || !lds_fits(k, lds_fr)) return FMX_ERR_UNSUPPORTED;
  if (F * D > 0x7fffffffll) { set_error("too many rows for one launch"); return FMX_ERR_UNSUPPORTED; }
  if (F * D == 0) return FMX_OK;
  int method = FMX_RANK_AVERAGE;
  FrIc ic{};
  FrZn zn{};
  const FrListLds ll = fr_list_lds(k, A, (size_t)fr_list_off(A, FR_CS_WORDS), 0);
  int lcap = ll.cap;
  void* args[] = {(void*)&X, (void*)&Yr, (void*)&D, (void*)&A, (void*)&ld, (void*)&method, (void*)&present,
                  (void*)&Yw, (void*)&qlo, (void*)&qhi, (void*)&RK, (void*)&ic, (void*)&zn, (void*)&lcap};
  FMX_HIP(set_dyn_lds(k, ll.bytes));
  FMX_HIP(hipLaunchKernel(k, fmx_grid2(D, F), dim3(nt_fa), args, ll.bytes, st));
  return FMX_OK;
}

}  // namespace fmx

BR_PHASE_EXPORT(fmx_debug_phase_cs)
