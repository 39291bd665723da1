// Order-independent exact summation of fp64 values in a fixed-point integer accumulator.
//
// The factor Gram that feeds the (discrete) correlation pruning is summed over per-date
// partials that live on different GPUs when the panel is date-sharded.  A floating-point
// sum depends on the order and grouping of its terms, so a 1-GPU and an 8-GPU run would
// round differently and a |C| near rho could flip the kept set.  Instead every partial is
// converted to a signed fixed-point number with LSB 2^-EX_FRAC (truncated toward zero,
// which is the same on every GPU count) held in EX_LIMBS limbs of 32 payload bits each,
// stored in int64 so that up to 2^31 terms add without a carry step.  Integer addition is
// associative: a rank's partial limbs, an RCCL all-reduce over ranks (any ring/tree order)
// and the final carry-normalisation give the same bits at 1, 2, 4 or 8 GPUs.
//
// Range: |x| < 2^(32 * EX_LIMBS - EX_FRAC - 1) = 2^127; smaller magnitudes than 2^-64 are
// dropped.  A non-finite or out-of-range term increments the flag limb, and the
// finalised value is then NaN (loud, not silently wrong).
#pragma once
#include <cstdint>

namespace fmx {

constexpr int EX_LIMBS = 6;            // payload limbs (32 bits each), little-endian
constexpr int EX_FRAC = 64;            // fixed-point fraction bits
constexpr int EX_SLOTS = EX_LIMBS + 1; // + the invalid-term flag

// Add x (truncated toward zero at 2^-EX_FRAC) into acc[0 .. EX_SLOTS).
__host__ __device__ inline void ex_add(int64_t* acc, double x) {
  union { double d; uint64_t u; } b;
  b.d = x;
  const uint64_t u = b.u;
  const bool neg = (u >> 63) != 0;
  const int ex = (int)((u >> 52) & 0x7ff);
  const uint64_t man = u & ((1ull << 52) - 1);
  if (ex == 0x7ff) { acc[EX_LIMBS] += 1; return; }    // inf / NaN
  uint64_t M;
  int E;
  if (ex == 0) { M = man; E = -1074; } else { M = man | (1ull << 52); E = ex - 1075; }
  if (M == 0) return;
  const int s = E + EX_FRAC;                           // x = M * 2^E = (M * 2^s) * 2^-EX_FRAC
  if (s + 53 > 32 * EX_LIMBS - 1) { acc[EX_LIMBS] += 1; return; }
#pragma unroll
  for (int k = 0; k < EX_LIMBS; ++k) {
    const int t = s - 32 * k;                          // chunk_k = floor(M * 2^t) mod 2^32
    uint64_t c;
    if (t >= 32 || t <= -64) c = 0;
    else if (t >= 0) c = (M << t) & 0xffffffffull;
    else c = (M >> (-t)) & 0xffffffffull;
    acc[k] += neg ? -(int64_t)c : (int64_t)c;
  }
}

// Carry-normalise (limbs 0..EX_LIMBS-2 into [0, 2^32), the top limb signed) and convert to
// double by Horner from the top limb down (fixed operation order: deterministic).
__host__ __device__ inline double ex_value(const int64_t* acc_in) {
  if (acc_in[EX_LIMBS] != 0) {
    union { uint64_t u; double d; } q;
    q.u = 0x7ff8000000000000ull;
    return q.d;
  }
  int64_t a[EX_LIMBS];
  int64_t carry = 0;
#pragma unroll
  for (int k = 0; k < EX_LIMBS - 1; ++k) {
    const int64_t v = acc_in[k] + carry;
    const int64_t lo = v & 0xffffffffll;
    carry = (v - lo) >> 32;                            // exact: v - lo is a multiple of 2^32
    a[k] = lo;
  }
  a[EX_LIMBS - 1] = acc_in[EX_LIMBS - 1] + carry;
  double r = (double)a[EX_LIMBS - 1];
#pragma unroll
  for (int k = EX_LIMBS - 2; k >= 0; --k) r = r * 4294967296.0 + (double)a[k];
  // * 2^-EX_FRAC (exact power-of-two scaling, no underflow for |r| >= 1 ulp of the grid)
  return r * 5.421010862427522170037264e-20;
}

}  // namespace fmx
