// Fine-bucket ranking of one row (fp64 keys) by one workgroup.
//
// Same contract as bucketrank.hpp -- the exact average rank
//     rank = #{y < x} + (#{y == x} + 1) / 2
// from bucket counts plus an in-bucket scan -- but the buckets are cut so that almost
// every element is alone in its bucket, which removes the in-bucket scan for most
// elements and the large block-wide splitter merge:
//
//  * one wave sorts a positional sample of 64 keys in registers (xor-shuffle bitonic);
//    the sorted samples s_0..s_{ns-1} plus the row's min and max cut the key space into
//    ns + 1 coarse intervals [min, s_0), [s_0, s_1), ..., [s_{ns-1}, max] holding
//    ~A/65 members each, and ns "equal to s_j" buckets that absorb heavy ties;
//  * inside coarse interval i an element lands in fine bucket
//        sub = min(K - 1, floor((x - lo_i) * (K / (hi_i - lo_i))))
//    Every step (IEEE subtract, multiply by a non-negative constant, floor, clamp) is
//    monotone non-decreasing in x and equal keys give equal results, so bucket ids are
//    monotone in the key: correctness never depends on how well the buckets are
//    balanced, only the cost of the in-bucket scan does.
//
// Bucket id layout (K+1 ids per interval): fine bucket sub of interval i is
// i*(K+1) + sub, the equal bucket of sample j is j*(K+1) + K, so ids increase with the
// key: I_0 fine, Eq(s_0), I_1 fine, Eq(s_1), ..., Eq(s_63), I_64 fine.
#pragma once

#include "bucketrank.hpp"

namespace fmx {

constexpr int FR_S = 64;   // samples = one wave
constexpr int FR_BEQ = 1 << 16;   // bucket-id flag of an equal-to-sample bucket (EQB searches)

// Lane index re-read at every call site: the persistent kernels loop over rows, and
// without this the compiler hoists every shuffle's lane-derived address (and the bitonic
// direction masks) out of the row loop into long-lived registers.
__device__ __forceinline__ int fr_lane() {
  int l = __lane_id();
  asm volatile("" : "+v"(l));
  return l;
}
// A value the compiler must treat as unknown at this point: per-element addresses are
// recomputed at their use (one VALU op) instead of being kept live across the kernel --
// the register allocator spills such address vectors rather than rematerialise them.
__device__ __forceinline__ int fr_opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ int fr_xor_i(int v, int m, int lane) {
  return __builtin_amdgcn_ds_bpermute((lane ^ m) << 2, v);
}
__device__ __forceinline__ double fr_xor_d(double v, int m, int lane) {
  const int a = (lane ^ m) << 2;
  const uint64_t u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)u);
  const int hi = __builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)(u >> 32));
  return __longlong_as_double((long long)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}
__device__ __forceinline__ uint64_t fr_xor_u64(uint64_t v, int m, int lane) {
  const int a = (lane ^ m) << 2;
  const int lo = __builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)v);
  const int hi = __builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)(v >> 32));
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
template <class T>
__device__ __forceinline__ T fr_up(T v, int o, int lane) {
  const int a = (lane - o) << 2;            // lanes < o read garbage; callers mask them
  if constexpr (sizeof(T) == 8) {
    const uint64_t u = (uint64_t)v;
    const int lo = __builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)u);
    const int hi = __builtin_amdgcn_ds_bpermute(a, (int)(uint32_t)(u >> 32));
    return (T)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
  } else {
    return (T)__builtin_amdgcn_ds_bpermute(a, (int)v);
  }
}

// 32-bit all-reduce over the 16 lanes of each DPP row (quad xor 1, xor 2, half-row
// mirror, row mirror): every lane ends with its row's result.
template <class Op>
__device__ __forceinline__ uint32_t fr_row_allreduce(uint32_t v, Op op) {
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false));
  v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false));
  return v;
}
// Wave-uniform min / max / sum of a 32-bit value (row all-reduce + 4 lane reads).
__device__ __forceinline__ uint32_t fr_wave_min_u32(uint32_t v) {
  auto op = [](uint32_t a, uint32_t b) { return a < b ? a : b; };
  v = fr_row_allreduce(v, op);
  return op(op(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
            op(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}
__device__ __forceinline__ uint32_t fr_wave_max_u32(uint32_t v) {
  auto op = [](uint32_t a, uint32_t b) { return a > b ? a : b; };
  v = fr_row_allreduce(v, op);
  return op(op(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
            op(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

// f64 DPP moves (two 32-bit halves) and wave sums: row all-reduce by quad xor 1, xor 2,
// half-row mirror, row mirror, then the four row totals through lane reads.  The
// summation order is fixed, so results are run-to-run deterministic.
template <int CTRL>
__device__ __forceinline__ double fr_dpp_d(double v) {
  const uint64_t u = __double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double fr_row_sum_d(double v) {
  v += fr_dpp_d<0xB1>(v);
  v += fr_dpp_d<0x4E>(v);
  v += fr_dpp_d<0x141>(v);
  v += fr_dpp_d<0x140>(v);
  return v;
}
__device__ __forceinline__ double fr_readlane_d(double v, int l) {
  const uint64_t u = __double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double fr_wave_sum_d(double v) {
  v = fr_row_sum_d(v);
  return (fr_readlane_d(v, 0) + fr_readlane_d(v, 16)) + (fr_readlane_d(v, 32) + fr_readlane_d(v, 48));
}
// A block-uniform double moved to SGPRs (frees two VGPRs for the rest of the kernel).
__device__ __forceinline__ double fr_uniform_d(double v) {
  const uint64_t u = __double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)u);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(u >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ uint64_t fr_readlane_u64(uint64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}

template <int CTRL>
__device__ __forceinline__ double fr_dpp_max_step(double v) {
  return fmax(v, fr_dpp_d<CTRL>(v));
}
// Block reduction without LDS shuffles (as br_part / br_fin): every wave reduces N values
// with DPP row all-reduces plus four lane reads, lane 0 parks them at scr[wid*S + off + i];
// fr_fin_dpp then combines the NT/64 wave results of value i < S (sum for i < nsum, max
// otherwise) into scr[(NT/64)*S + i].  scr: (NT/64 + 1) * S doubles.
template <int N, bool MAX>
__device__ __forceinline__ void fr_part_dpp(const double* v, double* scr, int S, int off) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double x = v[i];
    if (MAX) {
      x = fr_dpp_max_step<0xB1>(x);
      x = fr_dpp_max_step<0x4E>(x);
      x = fr_dpp_max_step<0x141>(x);
      x = fr_dpp_max_step<0x140>(x);
      x = fmax(fmax(fr_readlane_d(x, 0), fr_readlane_d(x, 16)), fmax(fr_readlane_d(x, 32), fr_readlane_d(x, 48)));
    } else {
      x = fr_row_sum_d(x);
      x = (fr_readlane_d(x, 0) + fr_readlane_d(x, 16)) + (fr_readlane_d(x, 32) + fr_readlane_d(x, 48));
    }
    if (lane == 0) scr[wid * S + off + i] = x;
  }
}
// Multi-value butterfly (same contract as fr_part_dpp, N in {2, 4, 8, 16}): each DPP
// exchange step halves the values a lane carries (it keeps one half, sends the other to
// its partner), so N values cost N-1 exchanges inside the 16-lane rows instead of 4N,
// then two cross-row swaps.  Lane bits 3..0 pick the half (row mirror, half-row mirror,
// quad xor 2, xor 1 are all involutions that flip those bits).
template <bool MAX>
__device__ __forceinline__ double fr_op2(double a, double b) { return MAX ? fmax(a, b) : a + b; }
template <int CTRL, int H, bool MAX>
__device__ __forceinline__ void fr_bfly_step(double* v, bool upper) {
#pragma unroll
  for (int i = 0; i < H; ++i) {
    const double send = upper ? v[i] : v[i + H];
    const double keep = upper ? v[i + H] : v[i];
    v[i] = fr_op2<MAX>(keep, fr_dpp_d<CTRL>(send));
  }
}
template <int N, bool MAX>
__device__ __forceinline__ void fr_part_bfly(const double* vin, double* scr, int S, int off) {
  static_assert(N == 2 || N == 4 || N == 8 || N == 16, "N");
  constexpr int LG = N == 2 ? 1 : N == 4 ? 2 : N == 8 ? 3 : 4;
  const int lane = fr_lane(), wid = threadIdx.x >> 6;
  double v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = vin[i];
  if constexpr (LG >= 4) fr_bfly_step<0x140, N / 2, MAX>(v, lane & 8);
  else v[0] = v[0];
  if constexpr (LG == 4) fr_bfly_step<0x141, N / 4, MAX>(v, lane & 4);
  if constexpr (LG == 4) fr_bfly_step<0x4E, N / 8, MAX>(v, lane & 2);
  if constexpr (LG == 4) fr_bfly_step<0xB1, N / 16, MAX>(v, lane & 1);
  if constexpr (LG == 3) {
    fr_bfly_step<0x140, 4, MAX>(v, lane & 8);
    fr_bfly_step<0x141, 2, MAX>(v, lane & 4);
    fr_bfly_step<0x4E, 1, MAX>(v, lane & 2);
    v[0] = fr_op2<MAX>(v[0], fr_dpp_d<0xB1>(v[0]));
  }
  if constexpr (LG == 2) {
    fr_bfly_step<0x140, 2, MAX>(v, lane & 8);
    fr_bfly_step<0x141, 1, MAX>(v, lane & 4);
    v[0] = fr_op2<MAX>(v[0], fr_dpp_d<0x4E>(v[0]));
    v[0] = fr_op2<MAX>(v[0], fr_dpp_d<0xB1>(v[0]));
  }
  if constexpr (LG == 1) {
    fr_bfly_step<0x140, 1, MAX>(v, lane & 8);
    v[0] = fr_op2<MAX>(v[0], fr_dpp_d<0x141>(v[0]));
    v[0] = fr_op2<MAX>(v[0], fr_dpp_d<0x4E>(v[0]));
    v[0] = fr_op2<MAX>(v[0], fr_dpp_d<0xB1>(v[0]));
  }
  // row r of the wave now holds, in lane 16r + j, its partial of value (j >> (4 - LG))
  double x = v[0];
  x = fr_op2<MAX>(x, fr_xor_d(x, 16, lane));
  x = fr_op2<MAX>(x, fr_xor_d(x, 32, lane));
  if (lane < 16 && (lane & ((16 >> LG) - 1)) == 0) scr[wid * S + off + (lane >> (4 - LG))] = x;
}

template <int NT>
__device__ __forceinline__ void fr_fin_dpp(double* scr, int S, int nsum) {
  constexpr int NR = NT / 64;
  const int t = threadIdx.x;
  __syncthreads();
  if (t < S) {
    double x = scr[t];
    for (int w = 1; w < NR; ++w) x = (t < nsum) ? x + scr[w * S + t] : fmax(x, scr[w * S + t]);
    scr[NR * S + t] = x;
  }
  __syncthreads();
}

// Value bounds from the high 32 bits of order keys: every key with high word in
// [hmin, hmax] has a value in [lo, hi] (NaN patterns of the synthetic keys -> +-inf).
__device__ __forceinline__ void fr_key_bounds(uint32_t hmin, uint32_t hmax, double* lo, double* hi) {
  double a = okey_inv((uint64_t)hmin << 32), b = okey_inv(((uint64_t)hmax << 32) | 0xffffffffull);
  *lo = (a == a) ? a : -INFINITY;
  *hi = (b == b) ? b : INFINITY;
}

// Block reduction partials (as br_part, with fresh lane addresses): wave-reduce N values
// (sum, or max when MAX) and park each wave's result at scr[wid*S + off + i].
template <int N, bool MAX>
__device__ __forceinline__ void fr_part(const double* v, double* scr, int S, int off) {
  const int lane = fr_lane(), wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double x = v[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const double y = fr_xor_d(x, o, lane);
      x = MAX ? fmax(x, y) : x + y;
    }
    if (lane == 0) scr[wid * S + off + i] = x;
  }
}

template <int K>
struct FRG {
  static constexpr int NB = (FR_S + 1) * (K + 1) - 1;   // bucket ids [0, NB)
};

// fr_build_w0's sample argument meaning "the samples are parked in T.spl" (a key that
// okey never produces: the NaN pattern's key sorts after +inf but before the sentinel).
constexpr uint64_t FR_FROM_LDS = 0xfffffffffffffffeull;

// LDS-resident cut of the key space.
struct FrTab {
  uint64_t spl[FR_S];        // sorted sample keys, KEY_SENTINEL-padded
  double2 li[FR_S + 1];      // interval (lower bound, K / (hi - lo) or 0 when the width
                             // is 0 / not finite): one 16-byte read per element
};


// Ascending bitonic sort of one key per lane across a wave (lane l ends with the l-th
// smallest); no LDS, no barrier.
__device__ __forceinline__ uint64_t wave_sort64(uint64_t v, int lane) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      const uint64_t o = fr_xor_u64(v, j, lane);
      const bool up = (lane & k) == 0;
      const bool lower = (lane & j) == 0;
      const uint64_t lo = v < o ? v : o, hi = v < o ? o : v;
      v = (lower == up) ? lo : hi;
    }
  }
  return v;
}

__device__ __forceinline__ double fr_inv(double lo, double hi, double kf) {
  const double w = hi - lo;
  double inv = (w > 0.0 && w < INFINITY) ? kf / w : 0.0;
  return (inv < INFINITY) ? inv : 0.0;
}

// Wave 0 only: sort the sample keys (one per lane) and fill the interval table.
// vmin / vmax bound every key that will be bucketed (a superset's bounds are fine).
template <int K>
__device__ void fr_build_w0(FrTab& T, uint64_t sample_key, double vmin, double vmax) {
  const int lane = fr_lane();
  // (a counting-rank sort of the parked samples -- each lane counting the samples below its
  // own from LDS broadcasts -- measured neutral in the fused pass and 2-7 % slower in the
  // ranks-only passes, where this sort is on the critical path: the shuffle network stays)
  const uint64_t s = wave_sort64(sample_key == FR_FROM_LDS ? T.spl[lane] : sample_key, lane);
  const uint64_t prev = fr_up(s, 1, lane);
  const int ns = __popcll(__ballot(s != KEY_SENTINEL));
  T.spl[lane] = s;
  const double kf = (double)K;
  double lo = 0.0, inv = 0.0;
  if (lane <= ns) {
    lo = lane == 0 ? vmin : okey_inv(prev);
    const double hi = lane == ns ? vmax : okey_inv(s);
    inv = fr_inv(lo, hi, kf);
  }
  T.li[lane] = make_double2(lo, inv);
  if (lane == 63) {                       // interval 64 exists only when ns == 64
    double lo64 = 0.0, inv64 = 0.0;
    if (ns == 64) {
      lo64 = okey_inv(s);
      inv64 = fr_inv(lo64, vmax, kf);
    }
    T.li[64] = make_double2(lo64, inv64);
  }
}

// Bucket id of a (non-sentinel) key with value v = okey_inv(key).
template <int K>
__device__ __forceinline__ int fr_bucket(const FrTab& T, uint64_t key, double v) {
  int i = 0;
#pragma unroll
  for (int step = 32; step >= 1; step >>= 1)
    if (T.spl[i + step - 1] <= key) i += step;
  const uint64_t last = T.spl[i];
  i += last <= key;                         // i = #samples <= key, in [0, 64]
  if (i > 0 && T.spl[i - 1] == key) return (i - 1) * (K + 1) + K;
  const double2 li = T.li[i];
  const double inv = li.y;
  const double t = (v - li.x) * inv;
  const int sub = inv > 0.0 ? (int)fmin(t, (double)(K - 1)) : 0;
  return i * (K + 1) + sub;
}

// Register sample: each of the NT/64 waves parks 64/(NT/64) of its keys in T.spl (lane j
// of wave w gives its element k = (j + w) % EMAX, row position w*64 + j + k*NT), so the
// 64 samples spread over every wave's columns and every register chunk at no memory
// cost.  Wave 0 sorts them in place after the next barrier (fr_build_w0 with from_lds).
template <int NT, int EMAX>
__device__ __forceinline__ void fr_park_sample(FrTab& T, const uint64_t* key) {
  constexpr int NW = NT / 64, PER = FR_S / NW;
  const int lane = fr_lane(), wid = threadIdx.x >> 6;
  if (lane < PER) {
    const int sel = (lane + wid) % EMAX;
    uint64_t v = KEY_SENTINEL;
#pragma unroll
    for (int k = 0; k < EMAX; ++k)
      if (k == sel) v = key[k];
    T.spl[wid * PER + lane] = v;
  }
}

// EQB: an equal-to-sample bucket id also carries FR_BEQ (callers mask it off for the counter)
template <int K, int G, bool EQB = false>
__device__ __forceinline__ void fr_bucket_grp(const FrTab& T, const uint64_t* key, int* b, int dummy) {
  int i[G];
  uint64_t last[G];                           // largest sample <= key
#pragma unroll
  for (int k = 0; k < G; ++k) i[k] = 0;
#pragma unroll
  for (int step = 32; step >= 1; step >>= 1) {
    uint64_t s[G];
#pragma unroll
    for (int k = 0; k < G; ++k) s[k] = T.spl[i[k] + step - 1];
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const bool c = s[k] <= key[k];
      i[k] += c ? step : 0;
    }
  }
  {
    uint64_t s[G];
#pragma unroll
    for (int k = 0; k < G; ++k) s[k] = T.spl[i[k]];
#pragma unroll
    for (int k = 0; k < G; ++k) {
      const bool c = s[k] <= key[k];
      i[k] += c ? 1 : 0;                      // #samples <= key
    }
  }
  double2 li[G];
#pragma unroll
  for (int k = 0; k < G; ++k) li[k] = T.li[i[k]];
#pragma unroll
  for (int k = 0; k < G; ++k) last[k] = T.spl[i[k] > 0 ? i[k] - 1 : 0];   // i == 0: never equal
#pragma unroll
  for (int k = 0; k < G; ++k) {
    const double tt = (okey_inv(key[k]) - li[k].x) * li[k].y;
    const int sub = li[k].y > 0.0 ? (int)fmin(tt, (double)(K - 1)) : 0;
    const int be = ((i[k] - 1) * (K + 1) + K) | (EQB ? FR_BEQ : 0), bf = i[k] * (K + 1) + sub;
    // a sentinel key (> every real key) only matches sentinel padding: dummy either way
    b[k] = key[k] == KEY_SENTINEL ? dummy : (last[k] == key[k] ? be : bf);
  }
}

// Bucket ids of all EMAX keys of a thread, searched in lockstep groups of up to 5 (that
// many independent LDS reads in flight per step) and branch-free; sentinel keys get
// bucket `dummy`.
// G: group size (fewer keys in flight for register-tight launches, e.g. 1024-thread rows
// at 64 VGPRs)
template <int K, int EMAX, int G = 4, bool EQB = false>
__device__ __forceinline__ void fr_bucket_all(const FrTab& T, const uint64_t* key, int* b, int dummy) {
  if constexpr (EMAX <= G + 1) {
    fr_bucket_grp<K, EMAX, EQB>(T, key, b, dummy);
  } else {
    fr_bucket_grp<K, G, EQB>(T, key, b, dummy);
    fr_bucket_all<K, EMAX - G, G, EQB>(T, key + G, b + G, dummy);
  }
}

// Positional sample of lane l: the element at the middle of the l-th of 64 equal strides
// (NaN / absent -> sentinel).
__device__ __forceinline__ uint64_t fr_sample(const double* x, const uint8_t* prow, int64_t A) {
  const int lane = fr_lane();
  const int64_t pos = ((int64_t)lane * A) / FR_S + A / (2 * FR_S);
  uint64_t sk = KEY_SENTINEL;
  if (pos < A && (prow ? prow[pos] != 0 : true)) {
    const double v = x[pos];
    if (v == v) sk = okey(v);
  }
  return sk;
}

// Packed 16-bit bucket counters: bucket b lives in half (b & 1) of word b >> 1.
__device__ __forceinline__ uint32_t fr_cnt_add(uint32_t* w, int b) {
  const uint32_t sh = (b & 1) << 4;
  return (atomicAdd(&w[b >> 1], 1u << sh) >> sh) & 0xffffu;
}
__device__ __forceinline__ uint32_t fr_cnt_get(const uint32_t* w, int b) {
  return (w[b >> 1] >> ((b & 1) << 4)) & 0xffffu;
}
// Counters b and b + 1 (after the scan: the bucket's start and end) from one ds_read2.
__device__ __forceinline__ void fr_cnt_get2(const uint32_t* w, int b, int* s0, int* s1) {
  const uint32_t* p = w + (b >> 1);
  const uint32_t w0 = p[0], w1 = p[1];
  const bool odd = b & 1;
  *s0 = (int)(odd ? (w0 >> 16) : (w0 & 0xffffu));
  *s1 = (int)(odd ? (w1 & 0xffffu) : (w0 >> 16));
}

// In-place exclusive scan of WORDS packed 16-bit counters (2 per word, 16-byte aligned),
// every thread owning a run of WORDS/NT consecutive words read and written as uint4.
// Exclusive starts stay below 65536 as long as the counted total (plus whatever sits in
// the last half-word) does.  scr: NT/64 ints.  Every thread must call it.
template <int NT, int WORDS>
__device__ void fr_scan16(uint32_t* w, int* scr) {
  constexpr int NW = NT / 64, R = WORDS / NT;
  static_assert(WORDS % (4 * NT) == 0, "run of whole uint4s");
  const int t = threadIdx.x, lane = fr_lane(), wid = t >> 6;
  uint4* v = reinterpret_cast<uint4*>(w) + t * (R / 4);
  auto sum4 = [](uint4 q) {
    return (int)((q.x & 0xffffu) + (q.x >> 16) + (q.y & 0xffffu) + (q.y >> 16) + (q.z & 0xffffu) + (q.z >> 16) +
                 (q.w & 0xffffu) + (q.w >> 16));
  };
  int loc = 0;
#pragma unroll
  for (int j = 0; j < R / 4; ++j) loc += sum4(v[j]);
  int incl = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = fr_up(incl, o, lane);
    if (lane >= o) incl += u;
  }
  if (lane == 63) scr[wid] = incl;
  __syncthreads();
  int base = 0;
#pragma unroll
  for (int x = 0; x < NW; ++x) base += (x < wid) ? scr[x] : 0;
  uint32_t run = (uint32_t)(base + incl - loc);
  auto ex = [&](uint32_t word) {
    const uint32_t lo = run, c0 = word & 0xffffu;
    const uint32_t hi = run + c0;
    run = hi + (word >> 16);
    return (lo & 0xffffu) | (hi << 16);
  };
#pragma unroll
  for (int j = 0; j < R / 4; ++j) {      // re-read: the run is not held in registers
    const uint4 q = v[j];
    uint4 o;
    o.x = ex(q.x); o.y = ex(q.y); o.z = ex(q.z); o.w = ex(q.w);
    v[j] = o;
  }
  __syncthreads();
}

// ---- List-balanced in-bucket scans ---------------------------------------------------
// An element sharing a fine bucket with other, distinct keys needs #less / #equal among the
// bucket's n members.  Scanned by its owning lane (one exec-masked loop per element slot),
// a wave pays max-over-lanes(n) iterations per slot while only ~40 % of its lanes have work.
// Instead every such element becomes a 32-bit work item (bucket start | slot << 16 | n << 24)
// in its WAVE's region of an LDS list; the wave walks its region with all lanes busy and the
// result (#less | #equal << 16) replaces the item.  Two kinds of item: pairs (n = 2: one
// compare with the other member, no loop) fill the region from the front, larger buckets
// (n <= 255) from the back, so consecutive items have similar work.  Claims are ballot
// prefix counts (no atomics, no cross-wave bases), the items are written while the counters
// are read, and the wave that claimed an item reads its result: no barrier of its own.
// Items that do not fit the region or have n > 255 are scanned by their owner (FR_SELF).
constexpr int FR_SELF = (int)0x80000000u;

struct FrClaim {
  int a = 0, b = 0;          // the wave's pair / multi items so far (wave-uniform)
};
// Claim (and write) the work item of one element slot across the wave.  items: the wave's
// region of wcap items.  Returns the item index | slot << 14, or slot | FR_SELF.  A slot's
// claims are all taken or all refused (region full), so the front and back never meet.
__device__ __forceinline__ int fr_claim_put(FrClaim& c, uint32_t* items, int wcap, bool scan, int n, int slot,
                                            int s0) {
  const bool pa = scan && n == 2, pb = scan && (unsigned)(n - 3) <= 252u;
  const uint64_t ma = __builtin_amdgcn_ballot_w64(pa), mb = __builtin_amdgcn_ballot_w64(pb);
  const int na = __popcll(ma), nb = __popcll(mb);
  const bool fits = c.a + na + c.b + nb <= wcap;        // wave-uniform
  // (a select of the whole mask and a ternary ref: the branch-free forms of both made the
  // compiler spill in the 80- and 128-VGPR rank kernels)
  const uint64_t m = pa ? ma : mb;
  const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  const int g = pa ? c.a + below : wcap - 1 - (c.b + below);
  if (fits) {
    c.a += na;
    c.b += nb;
  }
  const bool take = fits && (pa || pb);
  if (take) items[g] = (uint32_t)s0 | ((uint32_t)slot << 16) | ((uint32_t)n << 24);
  return take ? (g | slot << 14) : (slot | FR_SELF);
}
// The wave walks its own region: pairs [0, a), multis [wcap - b, wcap); result
// #less | #equal << 16 in place of each item, visible to the whole wave on return.
__device__ __forceinline__ void fr_list_walk_wave(const uint64_t* bkey, uint32_t* items, int wcap, const FrClaim& c) {
  const int lane = fr_lane();
  for (int g = lane; g < c.a; g += 64) {                // pairs: one compare
    const uint32_t it = items[g];
    const uint64_t* bk = bkey + (it & 0xffffu);
    const int slot = (int)((it >> 16) & 1u);
    const uint64_t own = bk[slot], oth = bk[slot ^ 1];
    items[g] = (uint32_t)((oth < own ? 1 : 0) + (oth == own ? 0x20000 : 0x10000));
  }
  for (int g = wcap - c.b + lane; g < wcap; g += 64) {  // two members per step: two reads in flight
    const uint32_t it = items[g];
    const uint64_t* bk = bkey + (it & 0xffffu);
    const int slot = (int)((it >> 16) & 0xffu), n = (int)(it >> 24);
    const uint64_t own = bk[slot];
    int acc = 0;
    for (int j = 0; j < n; j += 2) {
      const int j1 = j + 1 < n ? j + 1 : j;
      const uint64_t w0 = bk[j], w1 = bk[j1];
      acc += (w0 < own ? 1 : 0) + (w0 == own ? 0x10000 : 0);
      acc += j + 1 < n ? (w1 < own ? 1 : 0) + (w1 == own ? 0x10000 : 0) : 0;
    }
    items[g] = (uint32_t)acc;
  }
  // the wave's own LDS writes complete before any lane reads them back: lgkmcnt only (a
  // fence would also wait out vmcnt -- the persistent kernel's next-row loads in flight)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
// Scatter of a scanned element's key into its bucket range (after the counters are dead).
__device__ __forceinline__ void fr_scatter_key(uint64_t* bkey, int ref, int s0, uint64_t key) {
  const int slot = ref < 0 ? (ref & 0x3fff) : ((ref >> 14) & 0xff);
  bkey[s0 + slot] = key;
}
// Result of a scanned element: its item's, or its own scan when the list did not take it.
__device__ __forceinline__ int fr_result(const uint64_t* bkey, const uint32_t* items, int ref, int s0, int n) {
  if (ref >= 0) return (int)items[ref & 0x3fff];
  const uint64_t* bk = bkey + s0;
  const uint64_t own = bk[ref & 0x3fff];
  int acc = 0;
  for (int j = 0; j < n; ++j) {
    const uint64_t w = bk[j];
    acc += (w < own ? 1 : 0) + (w == own ? 0x10000 : 0);
  }
  return acc;
}
// Byte offset of the list behind the keys / counters (16-byte aligned).
__host__ __device__ inline int64_t fr_list_off(int64_t A, int64_t words) {
  const int64_t b = A * 8 > words * 4 ? A * 8 : words * 4;
  return (b + 15) / 16 * 16;
}

// In-place exclusive scan of c[0..n) with c[n] = total, by a block of NT threads (each
// owns a run of SC consecutive entries).  Every thread must call it.  scr: NT/64 Ts.
template <int NT, class T>
__device__ void fr_scan(T* c, int n, T* scr) {
  constexpr int NW = NT / 64;
  const int t = threadIdx.x, lane = fr_lane(), wid = t >> 6;
  const int sc = (n + 1 + NT - 1) / NT;
  const int b0 = t * sc;
  T loc = 0;
  for (int j = 0; j < sc; ++j)
    if (b0 + j < n) loc += c[b0 + j];
  T incl = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const T u = fr_up(incl, o, lane);
    if (lane >= o) incl += u;
  }
  if (lane == 63) scr[wid] = incl;
  __syncthreads();
  T base = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) base += (w < wid) ? scr[w] : (T)0;
  base += incl - loc;
  for (int j = 0; j < sc; ++j) {
    const int b = b0 + j;
    if (b < n) {
      const T x = c[b];
      c[b] = base;
      base += x;
    } else if (b == n) {
      c[b] = base;
    }
  }
  __syncthreads();
}

}  // namespace fmx
