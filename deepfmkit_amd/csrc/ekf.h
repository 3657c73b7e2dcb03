// ekf.h — per-sample Extended Kalman Filter (fitters.py:214-320), one lane per channel.
//
// The EKF is a serial chain over samples inside a channel (each update depends
// on the previous state), so the only parallelism is across independent
// channels/trials: lane = channel, the 5-vector state and the full 5×5
// covariance live in that lane's registers, and the sample loop runs in
// order. Operation order follows the numpy expressions of fitters.py:276-302:
//   P = F P F^T + Q (F = I: exact, so P + Q), H from fitters.py:287-293,
//   S = (H P) H^T + R, K = (P H^T) · (1/S), x += K y, P = (I − K H) P, the last
//   as P − K (H P) (below). sin / cos: the branch-free Cody-Waite form of
//   dfmi_math.h (library fallback for |x| >= 2^19).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfmi_math.h"

namespace dfmi {

__global__ __launch_bounds__(64) void ekf_kernel(const double* __restrict__ x, int64_t nrec, int64_t rec_stride,
                                                  int64_t n_samp, const double* __restrict__ x0,
                                                  const double* __restrict__ p0, const double* __restrict__ qd,
                                                  const double* __restrict__ rv, double w_m, double f_samp, int R,
                                                  int64_t nbuf, double* __restrict__ states) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrec) return;
  const double* __restrict__ xr = x + r * rec_stride;
  double st[5];
  double P[5][5];
  double Q[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    st[i] = x0[r * 5 + i];
    Q[i] = qd[i];
#pragma unroll
    for (int j = 0; j < 5; ++j) P[i][j] = (i == j) ? p0[i] : 0.0;
  }
  const double Rv = rv[r];
  // samples arrive 8 at a time (one 64-B load ahead of the chain that needs them);
  // the snapshot test counts down instead of a 64-bit modulo per sample
  int64_t to_snap = R;
  double xbuf[8];
  for (int64_t k = 0; k < n_samp; ++k) {
    const int slot = (int)(k & 7);
    if (slot == 0) {
#pragma unroll
      for (int u = 0; u < 8; ++u) xbuf[u] = (k + u < n_samp) ? xr[k + u] : 0.0;
    }
    double xk = xbuf[0];
#pragma unroll
    for (int u = 1; u < 8; ++u) xk = (slot == u) ? xbuf[u] : xk;
    // predict: P = F P F^T + Q with F = I
    // (off the diagonal numpy adds Q's exact zeros: a no-op unless P[i][j] is -0.0)
#pragma unroll
    for (int i = 0; i < 5; ++i) P[i][i] = P[i][i] + Q[i];
    const double a = st[0], m = st[1], phi = st[2], psi = st[3], dc = st[4];
    const double t = (double)k / f_samp;
    const double th = w_m * t + psi;
    double sth, cth;
    dfmi_sincos(th, &sth, &cth);
    const double arg = phi + m * cth;
    double sa, ca;
    dfmi_sincos(arg, &sa, &ca);
    const double h = a * ca + dc;
    double H[5] = {ca, -a * sa * cth, -a * sa, a * m * sa * sth, 1.0};
    const double y = xk - h;
    double HP[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int i = 0; i < 5; ++i) acc = fma(H[i], P[i][j], acc);
      HP[j] = acc;
    }
    double S = 0.0;
#pragma unroll
    for (int j = 0; j < 5; ++j) S = fma(HP[j], H[j], S);
    S = S + Rv;
    const double invS = 1.0 / S;
    double K[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < 5; ++j) acc = fma(P[i][j], H[j], acc);
      K[i] = acc * invS;
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) st[i] = st[i] + K[i] * y;
    // P = (I - K H) P  =  P - K (H P): the H P row formed for S above, 25 fma instead
    // of the literal 25 + 125 (states within 2e-15 of the literal form over 60k
    // samples, the size of the restated loop's own 1-ulp input sensitivity)
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = 0; j < 5; ++j) P[i][j] = fma(-K[i], HP[j], P[i][j]);
    if (--to_snap == 0) {
      to_snap = R;
      const int64_t b = (k + 1) / R - 1;
      if (b < nbuf) {
#pragma unroll
        for (int i = 0; i < 5; ++i) states[(r * nbuf + b) * 5 + i] = st[i];
      }
    }
  }
}

}  // namespace dfmi
