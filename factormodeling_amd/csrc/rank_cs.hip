// cs_rank launcher (bucket-rank kernels, rank_kernels.hpp).
// Reference: operations.py:54-62
#include "rank_launch.hpp"

namespace fmx {

fmx_status br_cs_rank(const double* X, double* Y, int64_t F, int64_t D, int64_t A, int64_t ld, int method,
                      const uint8_t* present, hipStream_t st) {
  void* args[] = {(void*)&X, (void*)&Y, (void*)&D, (void*)&A, (void*)&ld, (void*)&method, (void*)&present};
  const int nt = br_nt(1024);
  const size_t lds = (size_t)std::max<int64_t>(A, nt) * 8;
  return launch_br(FMX_EMAX_TABLE(k_cs_rank_br), nt, A, F * D, lds, args, st);
}

}  // namespace fmx

BR_PHASE_EXPORT(fmx_debug_phase_cs)
