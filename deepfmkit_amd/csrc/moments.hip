// moments.hip — np.mean / np.var of long float64 records on the device, bit-exact
// with numpy: EKFFitter.fit's two whole-record pre-reductions (/root/reference
// fitters.py:253 x[4] = np.mean(data), fitters.py:256 R_val = np.var(data)).
//
// numpy 2.x _methods._mean / _var: mean = umr_sum(arr) / n; var = umr_sum(x * x) / n
// with x = arr - mean, each elementwise step rounded on its own; umr_sum is the
// pairwise tree of np_sum.h (8-accumulator leaves of <= 128 elements, 8192-element
// buffer chunks chained left to right), planned on the host. The leaves in parallel
// straight from HBM (8 lanes per leaf, every record's leaves across the whole GPU), then
// one workgroup per record adds the tree's internal nodes level by level in LDS. This
// translation unit is compiled without FMA contraction, so (x - mean)^2 and the leaf
// additions round like numpy's.
#include "moments.h"

#include "np_sum.h"

namespace dfmi {
namespace {

constexpr int kT = 256;
// nodes (2 per leaf) the tree kernel keeps in static LDS: 16384 (128 KiB, records up to ~1M
// samples) fits gfx950's 160 KiB; the Makefile sets a smaller count for a 64-KiB-LDS ARCH
// (longer records then add the tree in the global node array)
#ifndef DFMI_TREE_LDS_NODES
#define DFMI_TREE_LDS_NODES 16384
#endif
constexpr int kTreeLds = DFMI_TREE_LDS_NODES;

// leaf element: a_i, or (a_i - mean)^2 rounded as numpy's x = arr - mean; x * x
template <bool SQ>
__device__ __forceinline__ double leaf_el(const double* a, int i, double mean) {
  if constexpr (SQ) {
    const double d = a[i] - mean;
    return d * d;
  } else {
    return a[i];
  }
}

// The plan's leaves (dfmi_np_leaf_sum over each), 8 lanes per leaf: lane j carries the
// leaf's accumulator r_j (elements j, j + 8, ... in order, as numpy's unrolled loop), the
// three shuffle levels add them as ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7)) (each
// add commutes, so every lane of a pair holds the same sum), lane 0 adds the tail. The
// 8 lanes of a leaf read 64 contiguous bytes per step: a record's leaves stream from HBM
// in parallel instead of one 1-KiB leaf per thread in sequence. grid (leaves / 32, nrec).
template <bool SQ>
__global__ __launch_bounds__(kT) void moments_leaf_kernel(const double* __restrict__ x, int64_t rec_stride,
                                                           const int* __restrict__ plan, int64_t nl,
                                                           double* __restrict__ nodes,
                                                           const double* __restrict__ mean, int64_t mean_stride) {
  const int64_t r = blockIdx.y;
  const int64_t t = (int64_t)blockIdx.x * kT + threadIdx.x;
  const int64_t leaf = t >> 3;
  const int j = (int)(t & 7);
  if (leaf >= nl) return;  // uniform over the leaf's 8 lanes
  const int* off = plan + 2;
  const int o = off[leaf], len = off[leaf + 1] - o;
  const double* a = x + r * rec_stride + o;
  const double m = SQ ? mean[r * mean_stride] : 0.0;
  double res;
  if (len < 8) {
    res = 0.0;
    for (int i = 0; i < len; ++i) res += leaf_el<SQ>(a, i, m);
  } else {
    const int e = len - (len % 8);
    double acc = leaf_el<SQ>(a, j, m);
    for (int i = 8 + j; i < e; i += 8) acc += leaf_el<SQ>(a, i, m);
    acc += __shfl_xor(acc, 1, 8);
    acc += __shfl_xor(acc, 2, 8);
    acc += __shfl_xor(acc, 4, 8);
    res = acc;
    for (int i = e; i < len; ++i) res += leaf_el<SQ>(a, i, m);
  }
  if (j == 0) nodes[r * 2 * nl + leaf] = res;
}

// The plan's internal nodes level by level (one workgroup per record; in LDS when the
// record's 2 nl nodes fit, else in the global node array), then root / n -> out.
template <bool LDS>
__global__ __launch_bounds__(kT) void moments_tree_kernel(const int* __restrict__ plan, int64_t nl,
                                                           double* __restrict__ nodes, int64_t n, double* out,
                                                           int64_t out_stride) {
  __shared__ double s[LDS ? kTreeLds : 1];
  const int64_t r = blockIdx.x;
  double* g = nodes + r * 2 * nl;
  double* v = LDS ? s : g;
  const int H = plan[1];
  const int* lvl = plan + 2 + nl + 1;
  const int* tri = lvl + H + 1;
  if (LDS) {
    for (int64_t t = threadIdx.x; t < nl; t += kT) v[t] = g[t];
    __syncthreads();
  }
  // the levels from hs on hold one node each (numpy's left-to-right chain over the 8192-sample
  // chunks: ~n / 8192 levels): one thread adds them in order without a barrier per level
  int hs = H;
  while (hs > 0 && lvl[hs] - lvl[hs - 1] == 1) --hs;
  for (int h = 0; h < hs; ++h) {
    for (int j = lvl[h] + threadIdx.x; j < lvl[h + 1]; j += kT) {
      const int* q = tri + 3 * j;
      v[q[0]] = v[q[1]] + v[q[2]];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    for (int j = lvl[hs]; j < lvl[H]; ++j) {
      const int* q = tri + 3 * j;
      v[q[0]] = v[q[1]] + v[q[2]];
    }
    out[r * out_stride] = v[nl > 1 ? 2 * nl - 2 : 0] / (double)n;
  }
}

}  // namespace

hipError_t moments_launch(const double* x, int64_t nrec, int64_t rec_stride, int64_t n, const int* plan,
                          int64_t n_leaves, double* nodes, double* mean, int64_t mean_stride, double* var,
                          int64_t var_stride, hipStream_t st) {
  if (nrec == 0) return hipSuccess;
  const dim3 lg((unsigned)((n_leaves * 8 + kT - 1) / kT), (unsigned)nrec);
  const bool lds = 2 * n_leaves <= kTreeLds;
  auto tree = [&](double* out, int64_t os) {
    if (lds)
      hipLaunchKernelGGL(moments_tree_kernel<true>, dim3((unsigned)nrec), dim3(kT), 0, st, plan, n_leaves, nodes, n,
                         out, os);
    else
      hipLaunchKernelGGL(moments_tree_kernel<false>, dim3((unsigned)nrec), dim3(kT), 0, st, plan, n_leaves, nodes, n,
                         out, os);
  };
  hipLaunchKernelGGL(moments_leaf_kernel<false>, lg, dim3(kT), 0, st, x, rec_stride, plan, n_leaves, nodes,
                     (const double*)nullptr, (int64_t)0);
  tree(mean, mean_stride);
  if (var) {
    hipLaunchKernelGGL(moments_leaf_kernel<true>, lg, dim3(kT), 0, st, x, rec_stride, plan, n_leaves, nodes,
                       (const double*)mean, mean_stride);
    tree(var, var_stride);
  }
  return hipGetLastError();
}

}  // namespace dfmi
