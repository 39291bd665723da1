// Launch plumbing shared by the bucket-rank translation units (rank_cs.hip,
// rank_q.hip, rank_ic.hip): row-length -> EMAX table, workgroup size choice.
#pragma once
#include <cstdlib>
#include <map>
#include <mutex>
#include "rank_kernels.hpp"

namespace fmx {

static inline int br_emax(int64_t A, int nt) {
  const int64_t e = ceil_div(std::max<int64_t>(A, 1), nt);
  static const int tab[] = {1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 20, 24, 32};
  for (int v : tab)
    if (e <= v && (int64_t)v * nt <= 16384) return v;
  return -1;
}

// Workgroup size of a row kernel: its measured best (cs_rank and the IC 1024, the quantile
// kernels 512 on MI355X at A = 5000), or FMX_BR_NT=512|1024 for all of them.
static inline int br_nt(int preferred) {
  static int forced = [] {
    const char* e = getenv("FMX_BR_NT");
    const int v = e ? atoi(e) : 0;
    return (v == 512 || v == 1024) ? v : 0;
  }();
  return forced ? forced : preferred;
}

// Row-rank implementation: fine buckets (finerank.hpp, default) or splitter buckets
// (bucketrank.hpp) with FMX_RANK_IMPL=br -- kept for A/B measurements.
enum { RANK_IMPL_FINE = 0, RANK_IMPL_BR = 1 };
static inline int rank_impl() {
  static int v = [] {
    const char* e = getenv("FMX_RANK_IMPL");
    return (e && e[0] == 'b' && e[1] == 'r') ? (int)RANK_IMPL_BR : (int)RANK_IMPL_FINE;
  }();
  return v;
}

// Static LDS bytes of kernel k, queried once per kernel (the hot rank launches ask on every
// step; the answer never changes: ADVICE r5).  -1 when the query fails.
static inline int64_t kern_static_lds(const void* k) {
  static std::mutex mu;
  static std::map<const void*, int64_t> cache;
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(k);
  if (it != cache.end()) return it->second;
  hipFuncAttributes at;
  const int64_t v = hipFuncGetAttributes(&at, k) == hipSuccess ? (int64_t)at.sharedSizeBytes : -1;
  cache.emplace(k, v);
  return v;
}

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) above the 64 KiB default, once per
// (kernel, size) high-water mark.
static inline hipError_t set_dyn_lds(const void* k, size_t bytes) {
  if (bytes <= 64 * 1024) return hipSuccess;
  static std::mutex mu;
  static std::map<const void*, size_t> done;
  std::lock_guard<std::mutex> g(mu);
  size_t& d = done[k];
  if (bytes <= d) return hipSuccess;
  const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess) d = bytes;
  return e;
}

// True when kernel k (static LDS) plus dyn bytes of dynamic LDS fit one CU's 160 KiB.
static inline bool lds_fits(const void* k, size_t dyn) {
  if (!k) return false;
  const int64_t st = kern_static_lds(k);
  return st >= 0 && (size_t)st + dyn <= 160 * 1024;
}

// Dynamic LDS of a fine-bucket rank launch with its in-bucket scan list (finerank.hpp
// fr_list_*): `base` bytes before the list (keys / counters, fr_list_off), then the list.  The
// capacity is as many 4-byte items as fit without lowering the rows per CU that the launch
// has without a list (static LDS + base + `extra`, the bytes other phases keep behind base),
// at most A: a row with more scanned elements than that scans the rest from their owners.
struct FrListLds {
  int cap;
  size_t bytes;
};
static inline FrListLds fr_list_lds(const void* k, int64_t A, size_t base, size_t extra) {
  const int64_t sl = k ? kern_static_lds(k) : -1;
  const size_t stat = sl > 0 ? (size_t)sl : 0;
  // per-workgroup LDS is allocated in granules (2 KiB assumed: LDS_Block_Size reports
  // multiples of it), so the rows per CU are counted on rounded sizes
  const size_t cu = 160 * 1024, gran = 2048;
  auto up = [&](size_t b) { return (b + gran - 1) / gran * gran; };
  const size_t need = up(stat + base + extra);
  const size_t rows = std::max<size_t>(1, cu / std::max<size_t>(need, 1));
  const size_t per = cu / rows / gran * gran;
  const size_t room = per > stat + base ? per - stat - base : 0;
  const int64_t cap = std::min<int64_t>(A, (int64_t)(room / 4) & ~3ll);
  FrListLds r;
  r.cap = (int)std::max<int64_t>(cap, 0);
  r.bytes = base + std::max<size_t>((size_t)r.cap * 4, extra);
  return r;
}

// rows = inner * outer blocks on a 2-D grid (fmx_grid2; the kernel reads its row as fmx_blk())
template <class K>
static inline fmx_status launch_br(K kern_table, int nt, int64_t A, int64_t inner, int64_t outer, size_t lds,
                                   void** args, hipStream_t st) {
  const void* k = kern_table(nt, br_emax(A, nt));
  if (!k) { set_error("row too long for the bucket-rank kernels (A > 16384)"); return FMX_ERR_UNSUPPORTED; }
  if (inner <= 0 || outer <= 0) return FMX_OK;
  if (inner * nt > 0xffffffffll || outer > 0x7fffffffll) { set_error("too many rows for one launch"); return FMX_ERR_UNSUPPORTED; }
  FMX_HIP(set_dyn_lds(k, lds));
  FMX_HIP(hipLaunchKernel(k, fmx_grid2(inner, outer), dim3(nt), args, lds, st));
  return FMX_OK;
}

// Launch of a persistent row kernel: as many workgroups as are co-resident on the
// device (occupancy x CUs), capped at the row count; the kernel walks the rows.
static inline fmx_status launch_persistent(const void* k, int nt, int64_t nrows, size_t lds, void** args,
                                           hipStream_t st) {
  if (!k) { set_error("row too long for the fine-bucket kernels"); return FMX_ERR_UNSUPPORTED; }
  if (nrows <= 0) return FMX_OK;
  FMX_HIP(set_dyn_lds(k, lds));
  static std::mutex mu;
  static std::map<std::pair<const void*, size_t>, int64_t> cache;
  int64_t slots;
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find({k, lds});
    if (it == cache.end()) {
      int dev = 0, cus = 0, per = 0;
      FMX_HIP(hipGetDevice(&dev));
      FMX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      FMX_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, nt, lds));
      it = cache.emplace(std::make_pair(k, lds), (int64_t)std::max(1, per) * std::max(1, cus)).first;
    }
    slots = it->second;
  }
  const int64_t grid = std::min<int64_t>(nrows, slots);
  FMX_HIP(hipLaunchKernel(k, dim3((unsigned)grid), dim3(nt), args, lds, st));
  return FMX_OK;
}

#define FMX_EMAX_CASES(KT, NT)                                               \
  switch (E) {                                                               \
    case 1: return (const void*)KT<NT, 1>;                                   \
    case 2: return (const void*)KT<NT, 2>;                                   \
    case 3: return (const void*)KT<NT, 3>;                                   \
    case 4: return (const void*)KT<NT, 4>;                                   \
    case 5: return (const void*)KT<NT, 5>;                                   \
    case 6: return (const void*)KT<NT, 6>;                                   \
    case 8: return (const void*)KT<NT, 8>;                                   \
    case 10: return (const void*)KT<NT, 10>;                                 \
    case 12: return (const void*)KT<NT, 12>;                                 \
    case 16: return (const void*)KT<NT, 16>;                                 \
    case 20: return (const void*)KT<NT, 20>;                                 \
    case 24: return (const void*)KT<NT, 24>;                                 \
    case 32: return (const void*)KT<NT, 32>;                                 \
    default: return (const void*)nullptr;                                    \
  }

// Workgroup size of the aliased-LDS cs_rank kernel for rows of A assets: 512 up to 8192
// assets, 1024 beyond (a row's keys fill half the CU's LDS there, so 16 waves per row
// instead of 8 -- C5's 10,000-asset rank pass: 287 -> 142 ms, profiles/r02/c5_h6.log).
// FMX_FA_NT=512|640|1024 forces one size.
static inline int fa_nt(int64_t A) {
  static int v = [] {
    const char* e = getenv("FMX_FA_NT");
    const int x = e ? atoi(e) : 0;
    return (x == 512 || x == 640 || x == 1024) ? x : 0;
  }();
  return v ? v : (A > 8192 ? 1024 : 512);
}

#define FMX_EMAX_TABLE3(KT)                                                  \
  [](int nt, int E) -> const void* {                                         \
    if (nt == 512) { FMX_EMAX_CASES(KT, 512) }                               \
    if (nt == 640) { FMX_EMAX_CASES(KT, 640) }                               \
    FMX_EMAX_CASES(KT, 1024)                                                 \
  }

#define FMX_EMAX_TABLE(KT)                                                   \
  [](int nt, int E) -> const void* {                                         \
    if (nt == 512) { FMX_EMAX_CASES(KT, 512) }                               \
    FMX_EMAX_CASES(KT, 1024)                                                 \
  }

}  // namespace fmx
