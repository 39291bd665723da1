// Shared device/host helpers for libfmx (MI355X / gfx950 factor-panel engine).
//
// Numerics contract: every kernel is compiled with -ffp-contract=off and without
// fast-math so that IEEE add/sub/mul/div/sqrt sequences reproduce the reference's
// pandas/numpy arithmetic bit-for-bit where the algorithm is replicated (rolling
// Kahan/Welford kernels, numpy pairwise sums, rank formulas, linear percentiles).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/fmx.h"

#define FMX_WAVE 64

namespace fmx {

void set_error(const std::string& msg);
fmx_status hip_check(hipError_t e, const char* what);

#define FMX_HIP(call)                                                        \
  do {                                                                       \
    hipError_t _e = (call);                                                  \
    if (_e != hipSuccess) return ::fmx::hip_check(_e, #call);                \
  } while (0)

#define FMX_ARG(cond, msg)                                                   \
  do {                                                                       \
    if (!(cond)) {                                                           \
      ::fmx::set_error(std::string("invalid argument: ") + (msg));           \
      return FMX_ERR_ARG;                                                    \
    }                                                                        \
  } while (0)

#define FMX_LAUNCH_CHECK(name) FMX_HIP(hipGetLastError())

__device__ __forceinline__ double qnan() { return __builtin_nan(""); }
__device__ __forceinline__ bool isnan_(double v) { return v != v; }

// Order-preserving unsigned key of a double (NaN never passed; -0.0 folded to +0.0
// so that pandas/scipy treat the two zeros as ties).
__device__ __forceinline__ uint64_t okey(double v) {
  v = (v == 0.0) ? 0.0 : v;
  uint64_t u = __double_as_longlong(v);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double okey_inv(uint64_t k) {
  uint64_t u = (k & 0x8000000000000000ull) ? (k & 0x7fffffffffffffffull) : ~k;
  return __longlong_as_double(u);
}
constexpr uint64_t KEY_SENTINEL = 0xffffffffffffffffull;  // sorts after +inf

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace fmx
