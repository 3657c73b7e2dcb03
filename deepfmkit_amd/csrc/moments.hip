// moments.hip — np.mean / np.var of long float64 records on the device, bit-exact
// with numpy: EKFFitter.fit's two whole-record pre-reductions (/root/reference
// fitters.py:253 x[4] = np.mean(data), fitters.py:256 R_val = np.var(data)).
//
// numpy 2.x _methods._mean / _var: mean = umr_sum(arr) / n; var = umr_sum(x * x) / n
// with x = arr - mean, each elementwise step rounded on its own; umr_sum is the
// pairwise tree of np_sum.h (8-accumulator leaves of <= 128 elements, 8192-element
// buffer chunks chained left to right), planned on the host. One workgroup per
// record: leaves in parallel straight from HBM, the tree's internal nodes level by
// level in a global workspace. This translation unit is compiled without FMA
// contraction, so (x - mean)^2 and the leaf additions round like numpy's.
#include "moments.h"

#include "np_sum.h"

namespace dfmi {
namespace {

constexpr int kT = 256;

// dfmi_np_leaf_sum over s_i = (a_i - mean) * (a_i - mean)
__device__ __forceinline__ double sq(const double* a, int i, double mean) {
  const double d = a[i] - mean;
  return d * d;
}

__device__ double leaf_sum_sq(const double* a, int n, double mean) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += sq(a, i, mean);
    return r;
  }
  double r0 = sq(a, 0, mean), r1 = sq(a, 1, mean), r2 = sq(a, 2, mean), r3 = sq(a, 3, mean);
  double r4 = sq(a, 4, mean), r5 = sq(a, 5, mean), r6 = sq(a, 6, mean), r7 = sq(a, 7, mean);
  int i = 8;
  const int e = n - (n % 8);
  for (; i < e; i += 8) {
    r0 += sq(a, i + 0, mean);
    r1 += sq(a, i + 1, mean);
    r2 += sq(a, i + 2, mean);
    r3 += sq(a, i + 3, mean);
    r4 += sq(a, i + 4, mean);
    r5 += sq(a, i + 5, mean);
    r6 += sq(a, i + 6, mean);
    r7 += sq(a, i + 7, mean);
  }
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (; i < n; ++i) res += sq(a, i, mean);
  return res;
}

// The plan's tree over x (SQ: over (x - mean)^2); every thread returns the root.
template <bool SQ>
__device__ double plan_sum(const double* __restrict__ x, const int* __restrict__ plan, double* nodes, double mean) {
  const int nl = plan[0], H = plan[1];
  const int* off = plan + 2;
  const int* lvl = off + nl + 1;
  const int* tri = lvl + H + 1;
  for (int t = threadIdx.x; t < nl; t += kT) {
    const int o = off[t], len = off[t + 1] - o;
    nodes[t] = SQ ? leaf_sum_sq(x + o, len, mean) : dfmi_np_leaf_sum(x + o, len);
  }
  __syncthreads();
  for (int h = 0; h < H; ++h) {
    for (int j = lvl[h] + threadIdx.x; j < lvl[h + 1]; j += kT) {
      const int* q = tri + 3 * j;
      nodes[q[0]] = nodes[q[1]] + nodes[q[2]];
    }
    __syncthreads();
  }
  const double s = nodes[nl > 1 ? 2 * nl - 2 : 0];
  __syncthreads();
  return s;
}

__global__ __launch_bounds__(kT) void moments_kernel(const double* __restrict__ x, int64_t rec_stride, int64_t n,
                                                      const int* __restrict__ plan, int64_t n_leaves, double* nodes,
                                                      double* mean, int64_t mean_stride, double* var,
                                                      int64_t var_stride) {
  const int64_t r = blockIdx.x;
  const double* xr = x + r * rec_stride;
  double* nr = nodes + r * 2 * n_leaves;
  const double m = plan_sum<false>(xr, plan, nr, 0.0) / (double)n;
  if (threadIdx.x == 0) mean[r * mean_stride] = m;
  if (var) {
    const double v = plan_sum<true>(xr, plan, nr, m) / (double)n;
    if (threadIdx.x == 0) var[r * var_stride] = v;
  }
}

}  // namespace

hipError_t moments_launch(const double* x, int64_t nrec, int64_t rec_stride, int64_t n, const int* plan,
                          int64_t n_leaves, double* nodes, double* mean, int64_t mean_stride, double* var,
                          int64_t var_stride, hipStream_t st) {
  if (nrec == 0) return hipSuccess;
  hipLaunchKernelGGL(moments_kernel, dim3((unsigned)nrec), dim3(kT), 0, st, x, rec_stride, n, plan, n_leaves, nodes,
                     mean, mean_stride, var, var_stride);
  return hipGetLastError();
}

}  // namespace dfmi
