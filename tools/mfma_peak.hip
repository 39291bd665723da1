// Achievable fp64 MFMA rate on this part: every wave runs CH independent
// v_mfma_f64_16x16x4f64 accumulator chains for ITER steps from registers (no LDS, no
// memory in the loop), WPS waves per SIMD.  Prints TF/s per (CH, waves/CU) so the Gram
// kernels' fractions can be read against a measured ceiling as well as the 78.6 TF spec.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_peak.hip -o tools/mfma_peak
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dbl4 __attribute__((ext_vector_type(4)));

template <int CH>
__global__ void k_peak(double* out, int iters, double seed) {
  dbl4 acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = dbl4{0.0, 0.0, 0.0, 0.0};
  double a = seed + threadIdx.x * 1e-9, b = seed - threadIdx.x * 1e-9;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int CH>
static void run(int threads, int blocks, int iters, double* out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  k_peak<CH><<<blocks, threads>>>(out, 16, 1.0);
  (void)hipEventRecord(e0);
  k_peak<CH><<<blocks, threads>>>(out, iters, 1.0);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double waves = (double)blocks * threads / 64;
  const double flops = waves * iters * CH * 16.0 * 16.0 * 4.0 * 2.0;
  printf("chains %2d  threads/WG %4d  WGs %5d  waves/CU %4.1f  %8.3f ms  %6.2f TF/s\n", CH, threads, blocks,
         waves / 256.0, ms, flops / (ms * 1e-3) / 1e12);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

int main() {
  double* out;
  (void)hipMalloc(&out, sizeof(double) * 4096 * 1024);
  const int iters = 20000;
  for (int wpc : {4, 8, 16}) {
    const int threads = 256, blocks = 256 * wpc / 4;
    run<1>(threads, blocks, iters, out);
    run<2>(threads, blocks, iters, out);
    run<4>(threads, blocks, iters, out);
    run<8>(threads, blocks, iters, out);
  }
  (void)hipFree(out);
  return 0;
}
