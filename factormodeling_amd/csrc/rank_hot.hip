// The step's two hot rank launchers in their own translation unit (quick rebuilds while
// tuning the fine-bucket kernels): the fused four-operator pass at C2 and the persistent
// ranks-only pass at C5.
// Reference: operations.py:54-86, :171-182; factor_selector.py:36-48.
#include "rank_fine.hpp"
#include "rank_launch.hpp"

namespace fmx {

template <int NT, int E> constexpr auto kcr_dense_h = k_cs_rank_fa<NT, E, false>;

// cs_rank + cs_winsor (+ doubled ranks) + cs_zscore + market_neutralize of dense rows in one
// pass (k_cs_rank_fa<ZN>); FMX_ERR_UNSUPPORTED when the row does not fit the fine kernel.
template <int NT, int E> constexpr auto kcrwz_dense = k_cs_rank_fa<NT, E, false, true, false, true>;
// Rows of dates [d0, d1) of every factor (the panel keeps its D dates; the kernel maps
// grid x to date d0 + x through pointers offset by d0 rows).
fmx_status br_cs_rank_winsor_zn(const double* X, double* Yr, double* Yw, double* Yz, double* Yn, int64_t F, int64_t D,
                                int64_t A, int64_t ld, int64_t d0, int64_t d1, double qlo, double qhi,
                                fmx_rank2_t* RK, PwTable pw, int slen, hipStream_t st) {
  const int nt_fa = fa_nt(A) == 1024 ? 1024 : 512;
  const size_t lds_fr = std::max<size_t>((size_t)A * 8, (size_t)FR_CS_WORDS * 4);
  const int E = br_emax(A, nt_fa);
  const void* k = E < 0 ? nullptr : FMX_EMAX_TABLE(kcrwz_dense)(nt_fa, E);
  // rows whose numpy moment tree is complete over 64 leaves (4097..8192 assets, e.g. C2's
  // 5000): the moments combine by shuffles, no serial wave-0 tree walk (block_pw_sum_t64)
  if (k && nt_fa == 512 && pw_tree64((int)A) && getenv("FMX_ZN_T64") == nullptr) {
    if (E == 10) k = (const void*)k_cs_rank_fa<512, 10, false, true, false, true, true>;
    else if (E == 12) k = (const void*)k_cs_rank_fa<512, 12, false, true, false, true, true>;
    else if (E == 16) k = (const void*)k_cs_rank_fa<512, 16, false, true, false, true, true>;
  }
  if (rank_impl() == RANK_IMPL_BR || !k || !lds_fits(k, lds_fr)) return FMX_ERR_UNSUPPORTED;
  if (F * D > 0x7fffffffll) { set_error("too many rows for one launch"); return FMX_ERR_UNSUPPORTED; }
  if (F * (d1 - d0) == 0) return FMX_OK;
  const int64_t off = d0 * ld;
  X += off; Yr += off; Yw += off; Yz += off; Yn += off;
  if (RK) RK += off;
  int method = FMX_RANK_AVERAGE;
  const uint8_t* present = nullptr;
  FrIc ic{};
  FrZn zn{Yz, Yn, pw, slen};
  // the moments' scratch sits where the scan list goes later
  const FrListLds ll = fr_list_lds(k, A, (size_t)fr_list_off(A, FR_CS_WORDS), FR_ZN_SCR_BYTES);
  int lcap = ll.cap;
  void* args[] = {(void*)&X, (void*)&Yr, (void*)&D, (void*)&A, (void*)&ld, (void*)&method, (void*)&present,
                  (void*)&Yw, (void*)&qlo, (void*)&qhi, (void*)&RK, (void*)&ic, (void*)&zn, (void*)&lcap};
  FMX_HIP(set_dyn_lds(k, ll.bytes));
  FMX_HIP(hipLaunchKernel(k, fmx_grid2(d1 - d0, F), dim3(nt_fa), args, ll.bytes, st));
  return FMX_OK;
}

// Doubled average ranks only (k_cs_rank_fa with Y = NULL): the rank pass a daily IC over
// raw factors starts from (fmx_ic_daily_ranked) when no operator output is wanted.
// Rows of 8193..10240 assets (C5): k_cs_rank_fa<1024, 10> at two rows per CU (its 80 KB of
// keys and a short scan list fit half the LDS; 64 VGPRs) -- 5.52 / 5.54 vs 6.03 / 6.03 ms per
// 126 dates x 500 factors for the persistent one-row-per-CU k_cs_rank2_pf (128 VGPRs, the
// next row's loads in flight; round 4's choice), profiles/r06/abM_*.log.  FMX_RANK2_PF=1
// keeps the persistent kernel for A/B.
static bool rank2_pf_enabled() {
  static const bool v = [] {
    const char* e = getenv("FMX_RANK2_PF");
    return e && e[0] == '1';
  }();
  return v;
}

fmx_status br_cs_rank2(const double* X, fmx_rank2_t* RK, int64_t F, int64_t D, int64_t A, int64_t ld, int64_t d0,
                       int64_t d1, hipStream_t st) {
  const int nt_fa = fa_nt(A) == 1024 ? 1024 : 512;
  const size_t lds_fr = std::max<size_t>((size_t)A * 8, (size_t)FR_CS_WORDS * 4);
  const int E = br_emax(A, nt_fa);
  const bool whole = d0 == 0 && d1 == D;      // the persistent kernel walks whole panels
  if (whole && nt_fa == 1024 && E == 10 && rank_impl() == RANK_IMPL_FINE && rank2_pf_enabled()) {
    int64_t nrows = F * D;
    const void* kp = (const void*)k_cs_rank2_pf<1024, 10>;
    const FrListLds ll = fr_list_lds(kp, A, (size_t)fr_list_off(A, FR_CS_WORDS), 0);
    int lcap = ll.cap;
    void* args[] = {(void*)&X, (void*)&nrows, (void*)&A, (void*)&ld, (void*)&RK, (void*)&lcap};
    return launch_persistent(kp, 1024, nrows, ll.bytes, args, st);
  }
  const void* k = E < 0 ? nullptr : FMX_EMAX_TABLE(kcr_dense_h)(nt_fa, E);
  if (!k || !lds_fits(k, lds_fr)) { set_error("fmx_cs_rank2: A <= 16384"); return FMX_ERR_UNSUPPORTED; }
  if (F * D > 0x7fffffffll) { set_error("too many rows for one launch"); return FMX_ERR_UNSUPPORTED; }
  if (F * (d1 - d0) == 0) return FMX_OK;
  X += d0 * ld;
  RK += d0 * ld;
  double* Y = nullptr;
  double* Y2 = nullptr;
  int method = FMX_RANK_AVERAGE;
  const uint8_t* present = nullptr;
  double qlo = 0.0, qhi = 0.0;
  FrIc ic{};
  FrZn zn{};
  const FrListLds ll = fr_list_lds(k, A, (size_t)fr_list_off(A, FR_CS_WORDS), 0);
  int lcap = ll.cap;
  void* args[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&method, (void*)&present,
                  (void*)&Y2, (void*)&qlo, (void*)&qhi, (void*)&RK, (void*)&ic, (void*)&zn, (void*)&lcap};
  FMX_HIP(set_dyn_lds(k, ll.bytes));
  FMX_HIP(hipLaunchKernel(k, fmx_grid2(d1 - d0, F), dim3(nt_fa), args, ll.bytes, st));
  return FMX_OK;
}

}  // namespace fmx
BR_PHASE_EXPORT(fmx_debug_phase_hot)
