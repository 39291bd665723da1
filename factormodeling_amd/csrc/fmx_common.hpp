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

// a / b, bit-identical to the IEEE quotient, for b > 0 normal with y = RN(1 / b) normal
// (a reciprocal table, a per-row reciprocal or a compile-time constant) and a quotient in
// the normal range.  q0 = RN(a y) is within 1.5 ulp of a / b; one fma
// correction (exact remainder e = a - q b) makes it faithful, and a second one rounds
// correctly (Markstein's theorem: y the correctly rounded reciprocal, q faithful).  Zero,
// very small, infinite and NaN dividends take the IEEE division instead (a branch that
// continuous data never takes).  1 mul + 4 fma at full rate, instead of the v_div_scale /
// quarter-rate v_rcp / v_div_fmas / v_div_fixup sequence and its hazard stalls.  Checked
// against the IEEE quotient on 3.4e8 random dividends x 68 divisors (tools/div_rn_check.c).
__device__ __forceinline__ double div_rn(double a, double b, double y) {
  double q = a * y;
  double e = __builtin_fma(-q, b, a);
  q = __builtin_fma(e, y, q);
  e = __builtin_fma(-q, b, a);
  q = __builtin_fma(e, y, q);
  const double m = __builtin_fabs(a);
  if (!(m >= 0x1p-900 && m <= 0x1.fffffffffffffp+1023)) q = a / b;
  return q;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace fmx
