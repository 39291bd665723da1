// Throughput of the VALU instruction classes the rank kernels lean on (development tool):
// each kernel runs a long chain of independent-ish ops per lane at full occupancy and
// reports cycles per wave-instruction per SIMD (from the kernel time, the CU count and the
// clock).  hipcc --offload-arch=gfx950 -O3 -o isa_rates isa_rates.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define N_IT 4096
#define UNR 16

__global__ void k_cmp_u64(const uint64_t* in, uint64_t* out) {
  uint64_t a[UNR];
  for (int u = 0; u < UNR; ++u) a[u] = in[threadIdx.x + u];
  uint64_t k = in[threadIdx.x + 100];
  int acc = 0;
  for (int it = 0; it < N_IT; ++it) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      acc += a[u] <= k ? 1 : 0;
      asm volatile("" : "+v"(a[u]));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
__global__ void k_cmp_u32(const uint64_t* in, uint64_t* out) {
  uint32_t a[UNR];
  for (int u = 0; u < UNR; ++u) a[u] = (uint32_t)in[threadIdx.x + u];
  uint32_t k = (uint32_t)in[threadIdx.x + 100];
  int acc = 0;
  for (int it = 0; it < N_IT; ++it) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      acc += a[u] <= k ? 1 : 0;
      asm volatile("" : "+v"(a[u]));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
__global__ void k_cmp_f64(const uint64_t* in, uint64_t* out) {
  double a[UNR];
  for (int u = 0; u < UNR; ++u) a[u] = (double)in[threadIdx.x + u];
  double k = (double)in[threadIdx.x + 100];
  int acc = 0;
  for (int it = 0; it < N_IT; ++it) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      acc += a[u] <= k ? 1 : 0;
      asm volatile("" : "+v"(a[u]));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}
__global__ void k_add_f64(const uint64_t* in, uint64_t* out) {
  double a[UNR];
  for (int u = 0; u < UNR; ++u) a[u] = (double)in[threadIdx.x + u];
  const double k = (double)in[threadIdx.x + 100];
  for (int it = 0; it < N_IT; ++it) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) a[u] = a[u] + k;
  }
  double s = 0;
  for (int u = 0; u < UNR; ++u) s += a[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}
__global__ void k_add_u32(const uint64_t* in, uint64_t* out) {
  uint32_t a[UNR];
  for (int u = 0; u < UNR; ++u) a[u] = (uint32_t)in[threadIdx.x + u];
  const uint32_t k = (uint32_t)in[threadIdx.x + 100];
  for (int it = 0; it < N_IT; ++it) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) a[u] = (a[u] + k) ^ (uint32_t)u;
  }
  uint32_t s = 0;
  for (int u = 0; u < UNR; ++u) s += a[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_cnd_u64(const uint64_t* in, uint64_t* out) {
  uint64_t a[UNR];
  for (int u = 0; u < UNR; ++u) a[u] = in[threadIdx.x + u];
  const uint64_t k = in[threadIdx.x + 100];
  const bool c = (threadIdx.x & 1) != 0;
  for (int it = 0; it < N_IT; ++it) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      a[u] = c ? a[u] : k;
      asm volatile("" : "+v"(a[u]));
    }
  }
  uint64_t s = 0;
  for (int u = 0; u < UNR; ++u) s += a[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_add_u64(const uint64_t* in, uint64_t* out) {
  uint64_t a[UNR];
  for (int u = 0; u < UNR; ++u) a[u] = in[threadIdx.x + u];
  const uint64_t k = in[threadIdx.x + 100];
  for (int it = 0; it < N_IT; ++it) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) a[u] = a[u] + k;
  }
  uint64_t s = 0;
  for (int u = 0; u < UNR; ++u) s ^= a[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*K)(const uint64_t*, uint64_t*);
int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  uint64_t *in, *out;
  hipMalloc(&in, 4096 * 8);
  hipMalloc(&out, (size_t)cus * 8 * 1024 * 8);
  hipMemset(in, 1, 4096 * 8);
  const char* names[] = {"cmp_u64(+add)", "cmp_u32(+add)", "cmp_f64(+add)", "add_f64", "add_u32+xor", "cnd_u64", "add_u64"};
  K ks[] = {k_cmp_u64, k_cmp_u32, k_cmp_f64, k_add_f64, k_add_u32, k_cnd_u64, k_add_u64};
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 7; ++i) {
    const int blocks = cus * 8, nt = 256;   // 8 waves per SIMD
    hipLaunchKernelGGL(ks[i], dim3(blocks), dim3(nt), 0, 0, in, out);
    hipEventRecord(a);
    hipLaunchKernelGGL(ks[i], dim3(blocks), dim3(nt), 0, 0, in, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double waves = (double)blocks * nt / 64;
    const double winstr = waves * N_IT * UNR;                   // wave-level ops (per the C source)
    const double simd_cycles = ms * 1e-3 * (clk * 1e3) * cus * 4;
    printf("%-16s %8.3f ms  %.2f SIMD-cycles per source op per wave\n", names[i], ms, simd_cycles / winstr);
  }
  return 0;
}
