// moments.h — launcher of the numpy-exact record moments (moments.hip), used by the
// C ABI in dfmi_capi.hip (dfmi_record_moments, dfmi_ekf_fit).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dfmi {

// np.mean(x_r) -> mean[r * mean_stride]; np.var(x_r) -> var[r * var_stride] (var may be
// null) for nrec records x_r = x[r * rec_stride .. + n], n >= 1. plan: the device copy
// of dfmi_pairwise_plan(n); nodes: nrec * plan[0] * 2 doubles of workspace.
hipError_t moments_launch(const double* x, int64_t nrec, int64_t rec_stride, int64_t n, const int* plan,
                          int64_t n_leaves, double* nodes, double* mean, int64_t mean_stride, double* var,
                          int64_t var_stride, hipStream_t st);

}  // namespace dfmi
