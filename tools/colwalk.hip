// Access-pattern probe for the time-series kernel family (development tool, not product
// code): each lane walks the dates of one (factor, asset) column of a [F][D][A] fp64
// panel -- the k_ts_reg / k_ts_set pattern -- reading X once and writing NOUT outputs.
// Variants: columns per lane (1: 8-B accesses, 2: 16-B), threads per block, and a plain
// grid-stride streaming copy as the HBM ceiling for the same read/write byte mix.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/colwalk tools/colwalk.hip && /tmp/colwalk
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));

template <int NOUT, int PF>
__global__ void __launch_bounds__(256) walk1(const double* __restrict__ X, double* __restrict__ Y, long F, long D,
                                             long A, long ld, long ostride) {
  const long col = (long)blockIdx.x * 256 + threadIdx.x;
  if (col >= F * A) return;
  const long f = col / A, a = col - f * A;
  const double* x = X + f * D * ld + a;
  double* y = Y + f * D * ld + a;
  double pf[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) pf[q] = x[q * ld];
  double acc = 0.0;
  for (long d = 0; d < D; d += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const double v = pf[q];
      if (d + q + PF < D) pf[q] = x[(d + q + PF) * ld];
      acc += v;
      if (d + q < D) {
#pragma unroll
        for (int o = 0; o < NOUT; ++o) y[o * ostride + (d + q) * ld] = acc * (double)(o + 1);
      }
    }
  }
}

template <int NOUT, int PF>
__global__ void __launch_bounds__(256) walk2(const double* __restrict__ X, double* __restrict__ Y, long F, long D,
                                             long A, long ld, long ostride) {
  const long A2 = A / 2;
  const long col = (long)blockIdx.x * 256 + threadIdx.x;
  if (col >= F * A2) return;
  const long f = col / A2, a = (col - f * A2) * 2;
  const dbl2* x = reinterpret_cast<const dbl2*>(X + f * D * ld + a);
  dbl2* y = reinterpret_cast<dbl2*>(Y + f * D * ld + a);
  const long l2 = ld / 2, o2 = ostride / 2;
  dbl2 pf[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) pf[q] = x[q * l2];
  dbl2 acc = {0.0, 0.0};
  for (long d = 0; d < D; d += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const dbl2 v = pf[q];
      if (d + q + PF < D) pf[q] = x[(d + q + PF) * l2];
      acc += v;
      if (d + q < D) {
#pragma unroll
        for (int o = 0; o < NOUT; ++o) y[o * o2 + (d + q) * l2] = acc * (double)(o + 1);
      }
    }
  }
}

// walk1 with nontemporal (streaming) stores for the outputs
template <int NOUT, int PF>
__global__ void __launch_bounds__(256) walk1nt(const double* __restrict__ X, double* __restrict__ Y, long F, long D,
                                               long A, long ld, long ostride) {
  const long col = (long)blockIdx.x * 256 + threadIdx.x;
  if (col >= F * A) return;
  const long f = col / A, a = col - f * A;
  const double* x = X + f * D * ld + a;
  double* y = Y + f * D * ld + a;
  double pf[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) pf[q] = __builtin_nontemporal_load(x + q * ld);
  double acc = 0.0;
  for (long d = 0; d < D; d += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const double v = pf[q];
      if (d + q + PF < D) pf[q] = __builtin_nontemporal_load(x + (d + q + PF) * ld);
      acc += v;
      if (d + q < D) {
#pragma unroll
        for (int o = 0; o < NOUT; ++o) __builtin_nontemporal_store(acc * (double)(o + 1), y + o * ostride + (d + q) * ld);
      }
    }
  }
}

// walk2 with nontemporal loads / stores
template <int NOUT, int PF>
__global__ void __launch_bounds__(256) walk2nt(const double* __restrict__ X, double* __restrict__ Y, long F, long D,
                                               long A, long ld, long ostride) {
  const long A2 = A / 2;
  const long col = (long)blockIdx.x * 256 + threadIdx.x;
  if (col >= F * A2) return;
  const long f = col / A2, a = (col - f * A2) * 2;
  const dbl2* x = reinterpret_cast<const dbl2*>(X + f * D * ld + a);
  dbl2* y = reinterpret_cast<dbl2*>(Y + f * D * ld + a);
  const long l2 = ld / 2, o2 = ostride / 2;
  dbl2 pf[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) pf[q] = __builtin_nontemporal_load(x + q * l2);
  dbl2 acc = {0.0, 0.0};
  for (long d = 0; d < D; d += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const dbl2 v = pf[q];
      if (d + q + PF < D) pf[q] = __builtin_nontemporal_load(x + (d + q + PF) * l2);
      acc += v;
      if (d + q < D) {
#pragma unroll
        for (int o = 0; o < NOUT; ++o) __builtin_nontemporal_store(acc * (double)(o + 1), y + o * o2 + (d + q) * l2);
      }
    }
  }
}

// walk2 with NT-thread blocks kept in lockstep (a barrier every PF dates), so that each
// date step of a block reads / writes NT * 16 contiguous bytes at about the same time
template <int NOUT, int PF, int NT>
__global__ void __launch_bounds__(NT) walk2s(const double* __restrict__ X, double* __restrict__ Y, long F, long D,
                                            long A, long ld, long ostride) {
  const long A2 = A / 2;
  const long col = (long)blockIdx.x * NT + threadIdx.x;
  const bool live = col < F * A2;
  const long f = live ? col / A2 : 0, a = live ? (col - f * A2) * 2 : 0;
  const dbl2* x = reinterpret_cast<const dbl2*>(X + f * D * ld + a);
  dbl2* y = reinterpret_cast<dbl2*>(Y + f * D * ld + a);
  const long l2 = ld / 2, o2 = ostride / 2;
  dbl2 pf[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q) pf[q] = live ? x[q * l2] : dbl2{0.0, 0.0};
  dbl2 acc = {0.0, 0.0};
  for (long d = 0; d < D; d += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const dbl2 v = pf[q];
      if (live && d + q + PF < D) pf[q] = x[(d + q + PF) * l2];
      acc += v;
      if (live && d + q < D) {
#pragma unroll
        for (int o = 0; o < NOUT; ++o) y[o * o2 + (d + q) * l2] = acc * (double)(o + 1);
      }
    }
    __syncthreads();
  }
}

template <int NOUT>
__global__ void __launch_bounds__(256) stream_copy(const dbl2* __restrict__ X, dbl2* __restrict__ Y, long n2,
                                                   long ostride2) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += (long)gridDim.x * 256) {
    const dbl2 v = X[i];
#pragma unroll
    for (int o = 0; o < NOUT; ++o) Y[o * ostride2 + i] = v * (double)(o + 1);
  }
}

template <class K>
static float timeit(K k, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  k();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) k();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const long F = 200, D = 2520, A = 5000, ld = A;
  const long n = F * D * ld;
  double *X, *Y;
  CK(hipMalloc(&X, n * 8));
  CK(hipMalloc(&Y, 5 * n * 8));
  CK(hipMemset(X, 0, n * 8));
  const double units = (double)F * D * A;
  auto rep = [&](const char* name, int nout, float ms) {
    printf("%-28s %8.3f ms  %7.1f GB/s\n", name, ms, (8.0 * (1 + nout)) * units / (ms * 1e-3) / 1e9);
  };
  const unsigned g1 = (unsigned)((F * A + 255) / 256), g2 = (unsigned)((F * A / 2 + 255) / 256);
  rep("walk1 out1 pf5", 1, timeit([&] { walk1<1, 5><<<g1, 256>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("walk1 out1 pf10", 1, timeit([&] { walk1<1, 10><<<g1, 256>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("walk2 out1 pf5", 1, timeit([&] { walk2<1, 5><<<g2, 256>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("walk1 out5 pf5", 5, timeit([&] { walk1<5, 5><<<g1, 256>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("walk2 out5 pf5", 5, timeit([&] { walk2<5, 5><<<g2, 256>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("walk2 out2 pf5", 2, timeit([&] { walk2<2, 5><<<g2, 256>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("walk1 out2 pf5", 2, timeit([&] { walk1<2, 5><<<g1, 256>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("walk2nt out5 pf5", 5, timeit([&] { walk2nt<5, 5><<<g2, 256>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("walk2nt out5 pf2", 5, timeit([&] { walk2nt<5, 2><<<g2, 256>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("walk1nt out5 pf5", 5, timeit([&] { walk1nt<5, 5><<<g1, 256>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("walk1nt out1 pf5", 1, timeit([&] { walk1nt<1, 5><<<g1, 256>>>(X, Y, F, D, A, ld, n); }, 3));
  auto g2s = [&](int nt) { return (unsigned)((F * A / 2 + nt - 1) / nt); };
  rep("walk2s out5 pf5 nt256", 5, timeit([&] { walk2s<5, 5, 256><<<g2s(256), 256>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("walk2s out5 pf5 nt1024", 5, timeit([&] { walk2s<5, 5, 1024><<<g2s(1024), 1024>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("walk2s out1 pf5 nt1024", 1, timeit([&] { walk2s<1, 5, 1024><<<g2s(1024), 1024>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("walk2s out5 pf10 nt1024", 5, timeit([&] { walk2s<5, 10, 1024><<<g2s(1024), 1024>>>(X, Y, F, D, A, ld, n); }, 3));
  rep("stream out1", 1, timeit([&] { stream_copy<1><<<4096, 256>>>((const dbl2*)X, (dbl2*)Y, n / 2, n / 2); }, 3));
  rep("stream out2", 2, timeit([&] { stream_copy<2><<<4096, 256>>>((const dbl2*)X, (dbl2*)Y, n / 2, n / 2); }, 3));
  rep("stream out5", 5, timeit([&] { stream_copy<5><<<4096, 256>>>((const dbl2*)X, (dbl2*)Y, n / 2, n / 2); }, 3));
  CK(hipFree(X));
  CK(hipFree(Y));
  return 0;
}
