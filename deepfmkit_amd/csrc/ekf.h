// ekf.h — per-sample Extended Kalman Filter (fitters.py:214-320), one lane per channel.
//
// The EKF is a serial chain over samples inside a channel (each update depends
// on the previous state), so the only parallelism is across independent
// channels/trials: lane = channel, the 5-vector state and the full 5×5
// covariance live in that lane's registers, and the sample loop runs in
// order. Operation order follows the numpy expressions of fitters.py:276-302:
//   P = F P F^T + Q (F = I: exact, so P + Q), H from fitters.py:287-293,
//   S = (H P) H^T + R, K = (P H^T) · (1/S), x += K y, P = (I − K H) P, the last
//   as P − K (H P) with P kept symmetric (ekf_step). sin / cos: the branch-free
//   Cody-Waite form of dfmi_math.h (library fallback for |x| >= 2^19); w_m t_k comes
//   from a parallel pre-pass, so the chain per sample is psi -> theta -> sincos ->
//   phase -> sincos -> H -> H P -> S -> 1/S -> K -> state.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dfmi_math.h"

namespace dfmi {

// theta's state-independent part, w_m * t_k with t_k = k / f_samp (np.arange(n) /
// f_samp, fitters.py:266; theta = w_m * t_axis[k] + psi, fitters.py:279): every sample
// in parallel, before the chain, so the chain adds psi only.
__global__ __launch_bounds__(256) void ekf_phase_kernel(double* __restrict__ wt, int64_t n, double w_m,
                                                        double f_samp) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) wt[k] = w_m * ((double)k / f_samp);
}

// One EKF step (fitters.py:274-302) on the lane's state; P symmetric: only its upper
// triangle P[i][j], i <= j, is read and written (constant-bound loops, fully unrolled:
// every index is a compile-time register).
// K = (P H^T) / S equals (H P)^T / S for a symmetric P: the H P row formed for S gives
// K, and P - K (H P) updates 15 entries (15 fma instead of 25 + 25 + 25; the
// reference's own P loses symmetry by rounding only).
__device__ __forceinline__ void ekf_step(double (&st)[5], double (&P)[5][5], const double (&Q)[5], double Rv,
                                         double xk, double wt) {
#pragma unroll
  for (int i = 0; i < 5; ++i) P[i][i] = P[i][i] + Q[i];  // predict: F = I
  const double a = st[0], m = st[1], phi = st[2], psi = st[3], dc = st[4];
  const double th = wt + psi;
  double sth, cth;
  dfmi_sincos(th, &sth, &cth);
  const double arg = phi + m * cth;
  double sa, ca;
  dfmi_sincos(arg, &sa, &ca);
  const double h = a * ca + dc;
  const double H[5] = {ca, -a * sa * cth, -a * sa, a * m * sa * sth, 1.0};
  const double y = xk - h;
  double HP[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) acc = fma(H[i], i <= j ? P[i][j] : P[j][i], acc);
    HP[j] = acc;
  }
  double S = 0.0;
#pragma unroll
  for (int j = 0; j < 5; ++j) S = fma(HP[j], H[j], S);
  S = S + Rv;
  // 1 / S (np.linalg.inv of the 1x1 S): v_rcp_f64 + two Newton steps, within an ulp
  double invS = __builtin_amdgcn_rcp(S);
  invS = fma(invS, fma(-S, invS, 1.0), invS);
  invS = fma(invS, fma(-S, invS, 1.0), invS);
  double K[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) K[i] = HP[i] * invS;
#pragma unroll
  for (int i = 0; i < 5; ++i) st[i] = st[i] + K[i] * y;
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j)
      if (j >= i) P[i][j] = fma(-K[i], HP[j], P[i][j]);
}

// wt: ekf_phase_kernel's w_m * t_k (n_samp values, shared by the channels).
__global__ __launch_bounds__(64) void ekf_kernel(const double* __restrict__ x, int64_t nrec, int64_t rec_stride,
                                                  int64_t n_samp, const double* __restrict__ x0,
                                                  const double* __restrict__ p0, const double* __restrict__ qd,
                                                  const double* __restrict__ rv, const double* __restrict__ wt, int R,
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
  // the snapshot test counts down (wave-uniform) instead of a 64-bit modulo per sample
  int64_t to_snap = R;
  auto snap = [&](int64_t k) {
    if (--to_snap == 0) {
      to_snap = R;
      const int64_t b = (k + 1) / R - 1;
      if (b < nbuf) {
#pragma unroll
        for (int i = 0; i < 5; ++i) states[(r * nbuf + b) * 5 + i] = st[i];
      }
    }
  };
  // samples and phases 8 at a time, the next group's loads in flight while the chain
  // runs the current one (unrolled: the sample slot is a compile-time index)
  int64_t k = 0;
  double xc[8], wc[8];
  const int64_t n8 = n_samp & ~(int64_t)7;
  if (n8 > 0) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xc[u] = xr[u];
      wc[u] = wt[u];
    }
  }
  for (; k < n8; k += 8) {
    double xn[8], wn[8];
    const bool more = k + 8 < n8;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xn[u] = more ? xr[k + 8 + u] : 0.0;
      wn[u] = more ? wt[k + 8 + u] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      ekf_step(st, P, Q, Rv, xc[u], wc[u]);
      snap(k + u);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xc[u] = xn[u];
      wc[u] = wn[u];
    }
  }
  for (; k < n_samp; ++k) {
    ekf_step(st, P, Q, Rv, xr[k], wt[k]);
    snap(k);
  }
}

}  // namespace dfmi
