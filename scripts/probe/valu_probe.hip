// Single-wave fp64 VALU issue/latency probe (gfx950): cycles per v_fma_f64 for 1, 2, 4
// and 8 independent dependency chains, and for an alternating fma/mul mix; s_memtime
// brackets (shader clock counter) in one wave. Used to decide whether the EKF / LM
// per-lane chains are latency- or issue-bound.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int CH>
__global__ void chains(double* out, long long* cyc, double a, double b, int iters) {
  double x[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) x[c] = threadIdx.x * 1e-3 + c;
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 64 / CH; ++u)
#pragma unroll
      for (int c = 0; c < CH; ++c) x[c] = fma(x[c], a, b);
  }
  long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += x[c];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  double* out;
  long long* cyc;
  hipMalloc(&out, 64 * 8);
  hipMalloc(&cyc, 8);
  const int iters = 4096;
  auto run = [&](auto kern, const char* name) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, out, cyc, 0.999999, 1e-9, iters);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, out, cyc, 0.999999, 1e-9, iters);
    long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("{\"probe\": \"%s\", \"cycles_per_fma\": %.3f}\n", name, (double)c / (64.0 * iters));
  };
  run(chains<1>, "fma_f64 1 chain");
  run(chains<2>, "fma_f64 2 chains");
  run(chains<4>, "fma_f64 4 chains");
  run(chains<8>, "fma_f64 8 chains");
  return 0;
}
