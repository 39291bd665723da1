// cs_rank launcher: fine-bucket kernels (rank_fine.hpp) by default, the splitter-bucket
// kernels (rank_kernels.hpp) with FMX_RANK_IMPL=br.
// Reference: operations.py:54-62
#include "rank_fine.hpp"
#include "rank_launch.hpp"

namespace fmx {

fmx_status br_cs_rank(const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld, int method,
                      const uint8_t* present, hipStream_t st) {
  void* args[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&method, (void*)&present};
  const int nt = br_nt(1024);
  const size_t lds_fr = (size_t)std::max<int64_t>(A, 1) * 8;
  auto fr_table = FMX_EMAX_TABLE(k_cs_rank_fr);
  if (rank_impl() == RANK_IMPL_BR || !lds_fits(fr_table(nt, br_emax(A, nt)), lds_fr)) {
    const size_t lds = (size_t)std::max<int64_t>(A, nt) * 8;
    return launch_br(FMX_EMAX_TABLE(k_cs_rank_br), nt, A, F * D, lds, args, st);
  }
  return launch_br(fr_table, nt, A, F * D, lds_fr, args, st);
}

}  // namespace fmx

BR_PHASE_EXPORT(fmx_debug_phase_cs)
