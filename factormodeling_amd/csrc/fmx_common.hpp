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

// Diagnostic (wrong-result) arms of the hot kernels exist for same-call A/B timing only
// (FR_DIAG_*, GDB_DIAG_*, GW_DIAG).  Each needs -DFMX_DIAG as well, and a translation unit
// built with FMX_DIAG registers itself at load time, so fmx_build_variant() names the
// library "diagnostic" and the Python loader refuses it unless FMX_ALLOW_DIAG=1.
#if !defined(FMX_DIAG) &&                                                                           \
    (defined(FR_DIAG_NOZNSUM) || defined(FR_DIAG_NOSCAN) || defined(FR_DIAG_NOPF) || defined(FR_DIAG_NOSTORE) || \
     defined(GDB_DIAG_NOSTAGE) || defined(CF_DIAG_RT) || defined(CF_DIAG_NOOLD) || (defined(GW_DIAG) && GW_DIAG != 0))
#error "diagnostic kernel arms need -DFMX_DIAG (and the library then loads only with FMX_ALLOW_DIAG=1)"
#endif
extern "C" void fmx_mark_diag(const char* tu);
#ifdef FMX_DIAG
namespace {
struct FmxDiagMark {
  FmxDiagMark() { fmx_mark_diag(__FILE__); }
} fmx_diag_mark_;
}  // namespace
#endif

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

// RN(x / n) for an integer n >= 1 from r = RN(1 / n) (a table entry): q0 = RN(x r) is within
// 1.5 ulp of x / n; the remainder x - q0 n is exact under an fma; q0 + r (x - q0 n) lies
// within 1.5 * 2^-53 ulp of x / n, which is never a rounding midpoint (x / n = odd * 2^(e-1)
// would need x to carry more than 53 bits) and sits at least ulp / (2n) away from one, so one
// fma rounding returns exactly the IEEE quotient (Markstein's correction).  3 fp64 ops in place
// of the ~10-instruction v_div_scale / v_rcp / Newton / v_div_fixup sequence.  Zero, tiny,
// huge and non-finite quotients take the IEEE divide (sign of zero, no under/overflow).
// The range guard reads q0's biased exponent with full-rate integer ops (fp64 compares
// issue at the quarter fp64 rate): exponents outside [64, 1958] (|q0| < 2^-959 incl. zero,
// |q0| >= 2^936, inf, NaN) take the divide.
__device__ __forceinline__ double mdiv(double x, double n, double r) {
  const double q0 = x * r;
  const uint32_t e = ((uint32_t)__double2hiint(q0) >> 20) & 0x7ffu;
  if (e - 64u > 1958u - 64u) return x / n;
  const double rem = __builtin_fma(-q0, n, x);
  return __builtin_fma(rem, r, q0);
}

// RN(x / b) for a GENERAL divisor b from r = RN(1 / b) (Markstein's theorem: r within 1/2 ulp
// of 1/b and q0 = RN(x r) within 1 ulp of x / b make rem = x - q0 b exact under an fma and
// RN(q0 + rem r) the correctly rounded quotient) -- for a row-uniform divisor such as a
// cross-sectional standard deviation, 3 fp64 ops per element in place of the IEEE divide
// sequence.  Range guards (integer tests of exponent fields): b_ok = rdiv_ok(b) keeps b in
// [2^-800, 2^800] (computed once per row); x below 2^-895 (zero included) and q0 outside
// [2^-959, 2^936] or non-finite take the IEEE divide -- no intermediate under/overflow.
// tests/native/rdiv_check.c: 1e8 host cases bit-identical to x / b.
__device__ __forceinline__ bool rdiv_ok(double b) {
  const uint32_t e = ((uint32_t)__double2hiint(b) >> 20) & 0x7ffu;
  return e - (1023u - 800u) <= 1600u;
}
__device__ __forceinline__ double rdiv(double x, double b, double r, bool b_ok) {
  const double q0 = x * r;
  const uint32_t eq = ((uint32_t)__double2hiint(q0) >> 20) & 0x7ffu;
  const uint32_t ex = ((uint32_t)__double2hiint(x) >> 20) & 0x7ffu;
  if (!b_ok || eq - 64u > 1958u - 64u || ex < 128u) return x / b;
  const double rem = __builtin_fma(-q0, b, x);
  return __builtin_fma(rem, r, q0);
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Row kernels launch their F * D (or D * F) rows as a 2-D grid dim3(inner, outer) and read
// the row as fmx_blk(): the work-items of ONE grid dimension are a 32-bit count, so a 1-D
// grid of rows x 1024 threads wraps past 4.19M rows (C4's 5.04M daily-IC rows ran only the
// first 846,000 -- the rest of the output was never written).
__device__ __forceinline__ int64_t fmx_blk() { return (int64_t)blockIdx.y * gridDim.x + blockIdx.x; }
inline dim3 fmx_grid2(int64_t inner, int64_t outer) { return dim3((unsigned)inner, (unsigned)outer); }

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

}  // namespace fmx
