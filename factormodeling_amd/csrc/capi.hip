// Library glue: error reporting, device info and the cached numpy pairwise-summation
// schedules used by the cross-sectional kernels.
#include <algorithm>
#include <array>
#include <map>
#include <mutex>
#include <vector>

#include "rowkit.hpp"

namespace fmx {

static thread_local std::string g_err;

void set_error(const std::string& msg) { g_err = msg; }

fmx_status hip_check(hipError_t e, const char* what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return FMX_ERR_HIP;
}

// ------------------------------------------------------------------------------------
// numpy pairwise summation tree (numpy/_core/src/umath/loops_utils.h.src, float64
// pairwise_sum): n < 8 -> sequential from 0; n <= 128 -> one 8-accumulator leaf;
// else split at n2 = n/2 rounded down to a multiple of 8 and recurse.  The ufunc
// reduction feeds the loop in 8192-element buffer chunks whose sums are added
// sequentially, so n > 8192 is a left-leaning chain of chunk trees.
struct Sched {
  std::vector<int32_t> lstart, llen;
  std::vector<int32_t> height;      // per node id (leaves 0..L-1 first)
  std::vector<int32_t> left, right; // per internal node (index k -> node L+k)
};

static int build_rec(int lo, int n, Sched& s, std::vector<std::array<int, 3>>& internals,
                     std::vector<int>& leaf_nodes, std::vector<int>& heights) {
  if (n <= 128) {
    s.lstart.push_back(lo);
    s.llen.push_back(n);
    int id = -(int)s.lstart.size();  // provisional negative id for leaves (1-based)
    return id;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  int l = build_rec(lo, n2, s, internals, leaf_nodes, heights);
  int r = build_rec(lo + n2, n - n2, s, internals, leaf_nodes, heights);
  internals.push_back({l, r, 0});
  return (int)internals.size() - 1;  // provisional non-negative id for internals
}

static std::vector<int32_t> build_schedule(int n) {
  std::vector<int32_t> out;
  if (n < 8) {
    out = {n, 0, 0, 0, 0};
    return out;
  }
  Sched s;
  std::vector<std::array<int, 3>> internals;
  std::vector<int> dummy1, dummy2;
  const int BUF = 8192;
  int root = build_rec(0, std::min(n, BUF), s, internals, dummy1, dummy2);
  for (int lo = BUF; lo < n; lo += BUF) {
    int c = build_rec(lo, std::min(BUF, n - lo), s, internals, dummy1, dummy2);
    internals.push_back({root, c, 0});
    root = (int)internals.size() - 1;
  }
  const int L = (int)s.lstart.size();
  const int I = (int)internals.size();
  auto final_id = [&](int prov) { return prov < 0 ? (-prov - 1) : (L + prov); };
  // heights (internals are created in post-order, children before parents)
  std::vector<int> h(L + I, 0);
  for (int k = 0; k < I; ++k) {
    int a = final_id(internals[k][0]), b = final_id(internals[k][1]);
    h[L + k] = 1 + std::max(h[a], h[b]);
  }
  int H = 0;
  for (int k = 0; k < I; ++k) H = std::max(H, h[L + k]);
  std::vector<int32_t> offs(H + 1, 0), trip;
  for (int r = 1; r <= H; ++r) {
    offs[r - 1] = (int32_t)(trip.size() / 3);
    for (int k = 0; k < I; ++k)
      if (h[L + k] == r) {
        trip.push_back(L + k);
        trip.push_back(final_id(internals[k][0]));
        trip.push_back(final_id(internals[k][1]));
      }
  }
  offs[H] = (int32_t)(trip.size() / 3);
  out.push_back(n);
  out.push_back(L);
  out.push_back(I);
  out.push_back(H);
  out.push_back(final_id(root));
  out.insert(out.end(), s.lstart.begin(), s.lstart.end());
  out.insert(out.end(), s.llen.begin(), s.llen.end());
  out.insert(out.end(), offs.begin(), offs.end());
  out.insert(out.end(), trip.begin(), trip.end());
  return out;
}

struct PwCache {
  int nmax = -1;
  int32_t* off = nullptr;
  int32_t* blob = nullptr;
};
static std::mutex g_pw_mu;
static std::map<int, PwCache> g_pw;  // per device

PwTable pw_table(int nmax, fmx_status* err) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  std::lock_guard<std::mutex> lk(g_pw_mu);
  PwCache& c = g_pw[dev];
  if (c.nmax < nmax) {
    int target = std::max(nmax, 1024);
    target = ((target + 1023) / 1024) * 1024;
    std::vector<int32_t> off(target + 1), blob;
    for (int n = 0; n <= target; ++n) {
      off[n] = (int32_t)blob.size();
      std::vector<int32_t> s = build_schedule(n);
      blob.insert(blob.end(), s.begin(), s.end());
    }
    int32_t *doff = nullptr, *dblob = nullptr;
    hipError_t e1 = hipMalloc((void**)&doff, sizeof(int32_t) * off.size());
    hipError_t e2 = hipMalloc((void**)&dblob, sizeof(int32_t) * blob.size());
    if (e1 != hipSuccess || e2 != hipSuccess) {
      *err = hip_check(e1 != hipSuccess ? e1 : e2, "hipMalloc(pairwise schedules)");
      return PwTable{nullptr, nullptr};
    }
    hipError_t e3 = hipMemcpy(doff, off.data(), sizeof(int32_t) * off.size(), hipMemcpyHostToDevice);
    hipError_t e4 = hipMemcpy(dblob, blob.data(), sizeof(int32_t) * blob.size(), hipMemcpyHostToDevice);
    if (e3 != hipSuccess || e4 != hipSuccess) {
      *err = hip_check(e3 != hipSuccess ? e3 : e4, "hipMemcpy(pairwise schedules)");
      return PwTable{nullptr, nullptr};
    }
    // old tables are intentionally kept alive: kernels already queued may still read them
    c.nmax = target;
    c.off = doff;
    c.blob = dblob;
  }
  return PwTable{c.off, c.blob};
}

}  // namespace fmx

using namespace fmx;

extern "C" const char* fmx_last_error(void) { return g_err.c_str(); }

extern "C" int32_t fmx_abi_version(void) { return FMX_ABI_VERSION; }

// Build variant: "product", or "diagnostic: <translation units>" when any unit was built
// with -DFMX_DIAG (fmx_common.hpp) -- such a library computes wrong results on purpose.
// (a function-local static: other units' load-time constructors may run before this one's)
static std::string& build_variant() {
  static std::string v = "product";
  return v;
}
extern "C" void fmx_mark_diag(const char* tu) {
  std::string& v = build_variant();
  v = (v == "product" ? std::string("diagnostic:") : v + ",") + " " + tu;
}
extern "C" const char* fmx_build_variant(void) { return build_variant().c_str(); }

extern "C" fmx_status fmx_device_info(char* buf, int64_t buflen) {
  FMX_ARG(buf && buflen > 0, "buffer");
  int dev = 0;
  FMX_HIP(hipGetDevice(&dev));
  hipDeviceProp_t p;
  FMX_HIP(hipGetDeviceProperties(&p, dev));
  snprintf(buf, (size_t)buflen, "%s cu=%d hbm=%zu clock_khz=%d", p.gcnArchName, p.multiProcessorCount,
           (size_t)p.totalGlobalMem, p.clockRate);
  return FMX_OK;
}

namespace fmx {
// Length (ints) of the schedule blob for n (cached; kernels stage short blobs in LDS).
int pw_len(int n) {
  static std::mutex mu;
  static std::map<int, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(n);
  if (it == cache.end()) it = cache.emplace(n, (int)build_schedule(n).size()).first;
  return it->second;
}
}  // namespace fmx

// Test hook: copy the schedule blob for n into out (host), returns its length.
// Every leaf of numpy's tree for n at depth 6 (64 leaves, one 8192-element chunk): the
// complete tree block_pw_sum_t64 combines by shuffles.
static bool leaves_at_depth(int n, int depth) {
  if (n <= 128) return depth == 0;
  if (depth == 0) return false;
  int n2 = n / 2;
  n2 -= n2 % 8;
  return leaves_at_depth(n2, depth - 1) && leaves_at_depth(n - n2, depth - 1);
}
bool fmx::pw_tree64(int n) { return n >= 8 && n <= 8192 && leaves_at_depth(n, 6); }

extern "C" int32_t fmx_debug_pw_schedule(int32_t n, int32_t* out, int32_t cap) {
  std::vector<int32_t> s = build_schedule(n);
  int32_t m = (int32_t)std::min<size_t>(s.size(), (size_t)cap);
  for (int32_t i = 0; i < m; ++i) out[i] = s[i];
  return (int32_t)s.size();
}
