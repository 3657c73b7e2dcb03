// diag.hip — dfmi_bessel_eval: the device Bessel code of the LM evaluated on a grid
// (diagnostics / GPU parity of row a14, scipy.special.jv at fit.py:106-108, 160,
// 275-276): the same device functions the fit kernels inline.
//   method 0: dfmi_bessel_table (dfmi_math.h: the general path's two-pass Miller walk)
//   method 1: bessel_regs<14>   (lm.h: the register path of ndata <= 12, one pass)
//   method 2: bessel_regs<18>   (lm.h: the register path of ndata <= 16)
// out[i*(nmax+1) + k] = J_k(x[i]).
#include <hip/hip_runtime.h>

#include "dfmi_math.h"
#include "lm.h"

namespace dfmi {

template <int NB>
__device__ void regs_row(double x, int nmax, double* o) {
  double J[NB];
  bessel_regs<NB>(x, NB - 1, J);
#pragma unroll
  for (int k = 0; k < NB; ++k)
    if (k <= nmax) o[k] = J[k];
}

__global__ __launch_bounds__(64) void bessel_eval_kernel(const double* __restrict__ x, int64_t nx, int nmax,
                                                         int method, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nx) return;
  double* o = out + i * (nmax + 1);
  if (method == 0) dfmi_bessel_table(x[i], nmax, o);
  else if (method == 1) regs_row<14>(x[i], nmax, o);
  else regs_row<18>(x[i], nmax, o);
}

hipError_t bessel_eval_launch(const double* x, int64_t nx, int nmax, int method, double* out, hipStream_t st) {
  if (nx <= 0) return hipSuccess;
  hipLaunchKernelGGL(bessel_eval_kernel, dim3((unsigned)((nx + 63) / 64)), dim3(64), 0, st, x, nx, nmax, method,
                     out);
  return hipGetLastError();
}

}  // namespace dfmi
