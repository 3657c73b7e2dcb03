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
//   Cody-Waite form of dfmi_math.h with its constants in SGPRs (dfmi_sincos_k; library
//   patch for |x| >= 2^19); w_m t_k comes from a parallel pre-pass, so the chain per
//   sample is psi -> theta -> sincos -> phase -> sincos -> H -> H P -> S -> 1/S -> state.
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

// x0 = [init4, NaN] and r_val per record for dfmi_ekf_fit (the mean and, without a given
// r_val, the variance are written by the moments kernels after this): init4 / r_val from
// device pointers when given (no host round trip), else from the by-value copies.
struct EkfInit {
  double i4[4];
  double rv;
};
__global__ __launch_bounds__(64) void ekf_x0_kernel(double* __restrict__ x0, double* __restrict__ rv, int64_t nrec,
                                                    const double* __restrict__ i4p, const double* __restrict__ rvp,
                                                    bool have_rv, EkfInit hv) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrec) return;
#pragma unroll
  for (int i = 0; i < 4; ++i) x0[r * 5 + i] = i4p ? i4p[i] : hv.i4[i];
  x0[r * 5 + 4] = __builtin_nan("");
  rv[r] = !have_rv ? __builtin_nan("") : rvp ? rvp[0] : hv.rv;
}

// One EKF step (fitters.py:274-302) on the lane's state; P symmetric: only its upper
// triangle P[i][j], i <= j, is read and written (constant-bound loops, fully unrolled:
// every index is a compile-time register).
// K = (P H^T) / S equals (H P)^T / S for a symmetric P: the H P row formed for S gives
// K, and P - K (H P) updates 15 entries (15 fma instead of 25 + 25 + 25; the
// reference's own P loses symmetry by rounding only).
// One wave runs one instruction stream whether its chains are dependent or not (a
// single wave issues a dependent v_fma_f64 every ~5.4 clocks, as fast as independent
// ones: profiles/r02l_valu_probe.jsonl), so the step is costed in instructions: H[4] = 1
// starts each H P chain at P[4][j], R folds into S, 1/S takes one Newton step on
// v_rcp_f64 (~1 ulp), phi + m cos(theta) is one fma. Every change is a rounding-order
// change against numpy's expressions (the reference itself moves by ~1e-15 under 1-ulp
// changes; tests/test_gpu_parity.py holds the kernel to 1e-12 of the oracle).
// ekf_step that also hands out the measurement row H and h = h(x) at the predicted state
// (the EKF parallel in time folds the sample's linearized element from them, ekf_pit.h)
__device__ __forceinline__ void ekf_step_h(double (&st)[5], double (&P)[5][5], const double (&Q)[5], double Rv,
                                           double xk, double wt, const DfmiTrigK& tk, double (&H)[5], double& h);
__device__ __forceinline__ void ekf_step(double (&st)[5], double (&P)[5][5], const double (&Q)[5], double Rv,
                                         double xk, double wt, const DfmiTrigK& tk) {
  double H[5], h;
  ekf_step_h(st, P, Q, Rv, xk, wt, tk, H, h);
}
__device__ __forceinline__ void ekf_step_h(double (&st)[5], double (&P)[5][5], const double (&Q)[5], double Rv,
                                           double xk, double wt, const DfmiTrigK& tk, double (&H)[5], double& h) {
#pragma unroll
  for (int i = 0; i < 5; ++i) P[i][i] = P[i][i] + Q[i];  // predict: F = I
  const double a = st[0], m = st[1], phi = st[2], psi = st[3], dc = st[4];
  const double th = wt + psi;
  double sth, cth;
  dfmi_sincos_k(th, tk, &sth, &cth);
  const double arg = fma(m, cth, phi);
  const double acth = -a * cth, amsth = (a * m) * sth;
  double sa, ca;
  dfmi_sincos_k(arg, tk, &sa, &ca);
  h = fma(a, ca, dc);
  H[0] = ca;
  H[1] = acth * sa;
  H[2] = -a * sa;
  H[3] = amsth * sa;
  H[4] = 1.0;
  const double y = xk - h;
  auto Pu = [&](int i, int j) -> double { return i <= j ? P[i][j] : P[j][i]; };
  double HP[5];
#pragma unroll
  for (int j = 0; j < 5; ++j)  // H[4] = 1: the chain starts from P[4][j]
    HP[j] = fma(H[3], Pu(3, j), fma(H[2], Pu(2, j), fma(H[1], Pu(1, j), fma(H[0], Pu(0, j), Pu(4, j)))));
  const double S = fma(HP[3], H[3], fma(HP[2], H[2], fma(HP[1], H[1], fma(HP[0], H[0], HP[4] + Rv))));
  // 1 / S (np.linalg.inv of the 1x1 S): v_rcp_f64 + one Newton step
  double invS = __builtin_amdgcn_rcp(S);
  invS = fma(invS, fma(-S, invS, 1.0), invS);
  const double iy = invS * y;
  double K[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) K[i] = HP[i] * invS;
#pragma unroll
  for (int i = 0; i < 5; ++i) st[i] = fma(HP[i], iy, st[i]);
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
                                                  int64_t nbuf, double* __restrict__ states, DfmiTrigK tk,
    const int* __restrict__ idx) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrec) return;
  // idx (optional): channel r of this launch is record idx[r] of the caller's arrays
  const int64_t rid = idx ? (int64_t)idx[r] : r;
  const double* __restrict__ xr = x + rid * rec_stride;
  double st[5];
  double P[5][5];
  double Q[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    st[i] = x0[rid * 5 + i];
    Q[i] = qd[i];
#pragma unroll
    for (int j = 0; j < 5; ++j) P[i][j] = (i == j) ? p0[i] : 0.0;
  }
  const double Rv = rv[rid];
  // the snapshot test counts down (wave-uniform) instead of a 64-bit modulo per sample
  int64_t to_snap = R;
  auto snap = [&](int64_t k) {
    if (--to_snap == 0) {
      to_snap = R;
      const int64_t b = (k + 1) / R - 1;
      if (b < nbuf) {
#pragma unroll
        for (int i = 0; i < 5; ++i) states[(rid * nbuf + b) * 5 + i] = st[i];
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
    // the next group, unconditionally (clamped into the record: no branch per load)
    const int64_t kn = k + 8 < n8 ? k + 8 : k;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xn[u] = xr[kn + u];
      wn[u] = wt[kn + u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      ekf_step(st, P, Q, Rv, xc[u], wc[u], tk);
      snap(k + u);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xc[u] = xn[u];
      wc[u] = wn[u];
    }
  }
  for (; k < n_samp; ++k) {
    ekf_step(st, P, Q, Rv, xr[k], wt[k], tk);
    snap(k);
  }
}

// ---------------------------------------------------------------------------
// Row-per-channel EKF (few channels): one 16-lane DPP row per channel, 4 channels per
// wave. Lane j < 5 of a row owns COLUMN j of the covariance (lanes 5..15 duplicate
// column 4); the state, theta, the sincos pair and H are computed by every lane of the
// row (one instruction stream costs the same for 1 or 16 lanes). Per sample the row
// then needs H P as one 5-fma chain per lane instead of 20 in one lane, one
// row_newbcast per H P element to share it, and a 5-fma column update instead of 15:
// ~100 wave instructions per sample against ~170 for ekf_step, which runs the same
// per-channel chain in one lane (the single-lane chain is issue-bound, see ekf_step).
// Same expressions as ekf_step (same fma chains, same 1/S), except the covariance
// update P[i][j] - HP_i (HP_j / S) where ekf_step forms (HP_i / S) HP_j: rounding only.
// ---------------------------------------------------------------------------

// value of lane n of this lane's 16-lane row, 64 bits in one v_mov_b64_dpp (gfx950's
// 64-bit DPP takes row_newbcast): the same bits as two 32-bit moves. `old` is the DPP
// instruction's tied destination, never read (all rows and banks enabled): passing a
// register whose value is dead (the previous sample's result) saves the copy the
// compiler otherwise makes to give every result its own destination.
template <int N>
__device__ __forceinline__ double row_bcast64(double old, double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const long long o = __builtin_bit_cast(long long, old);
  return __builtin_bit_cast(double, (long long)__builtin_amdgcn_update_dpp(o, b, 0x150 + N, 0xF, 0xF, false));
}

// Per-lane kernel-polynomial coefficients of dfmi_sincos_k (z^5 .. z^0) for the row
// sincos below: the sin kernel's on even lanes, the cos kernel's on odd lanes.
struct RowSplitCoef {
  double k[6];
};
__device__ __forceinline__ RowSplitCoef row_split_coef(const DfmiTrigK& k, int par) {
  RowSplitCoef rc;
#pragma unroll
  for (int i = 0; i < 6; ++i) rc.k[i] = par ? k.c[10 + i] : k.c[4 + i];
  return rc;
}

// dfmi_sincos_k(x) for a 16-lane row whose lanes all hold the same x, same bits: even
// lanes evaluate the sin kernel fma(r z, P_s, r), odd lanes the cos kernel
// fma(z z, P_c, fma(-0.5, z, 1)) (one polynomial per lane instead of both), every lane
// reads both back from lanes 0 and 1 of its row, and the quadrant is applied as in
// dfmi_sincos_k (swap selects + sign flips). ~31 VALU instructions instead of ~41.
__device__ __forceinline__ void ekf_sincos_row(double x, const DfmiTrigK& k, const RowSplitCoef& rc, bool odd,
                                               double& sn, double& cs) {
  const double q = rint(x * k.c[0]);
  double r = fma(-q, k.c[1], x);
  r = fma(-q, k.c[2], r);
  r = fma(-q, k.c[3], r);
  const double z = r * r;
  const double P = fma(z, fma(z, fma(z, fma(z, fma(z, rc.k[0], rc.k[1]), rc.k[2]), rc.k[3]), rc.k[4]), rc.k[5]);
  const double X = odd ? z : r;
  const double Y = odd ? fma(-0.5, z, 1.0) : r;
  const double v = fma(X * z, P, Y);
  const double sr = row_bcast64<0>(sn, v), cr = row_bcast64<1>(cs, v);
  const int qi = ((int)q) & 3;
  const double a = (qi & 1) ? cr : sr;
  const double b = (qi & 1) ? sr : cr;
  sn = (qi & 2) ? -a : a;
  cs = ((qi + 1) & 2) ? -b : b;
  if (__builtin_expect(!(fabs(x) < 524288.0), 0)) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double2 w = dfmi_sincos_lib(x);
    sn = w.x;
    cs = w.y;
#endif
  }
}

// Registers the row step keeps across samples: the DPP results (their previous values are
// the tied destinations of the next sample's moves) and the one-channel coefficients.
struct RowRegs {
  double HP[5];
  double sth, cth, sa, ca;
};

// SPLIT: both sincos by ekf_sincos_row; otherwise dfmi_sincos_k per lane (same bits; A/B
// builds). The chain is fp64-issue-bound, not latency-bound: a form with 8 fewer dependent
// steps per sample (Estrin polynomials, (H P)_j and S as shallow trees, the Newton step of
// 1/S folded into iy and K_j) but 5 more fp64 instructions ran 3 % slower
// (profiles/r03j_ekf_modes_ab.json).
template <bool SPLIT>
__device__ __forceinline__ void ekf_row_step(double (&st)[5], double (&Pc)[5], const double (&qv)[5], double Rv,
                                             double xk, double wt, const DfmiTrigK& tk, RowRegs& rr,
                                             const RowSplitCoef& rc, bool odd) {
#pragma unroll
  for (int i = 0; i < 5; ++i) Pc[i] = Pc[i] + qv[i];  // predict: Q on the diagonal (qv[i] = 0 off it)
  const double a = st[0], m = st[1], phi = st[2], psi = st[3], dc = st[4];
  const double th = wt + psi;
  if constexpr (SPLIT) ekf_sincos_row(th, tk, rc, odd, rr.sth, rr.cth);
  else dfmi_sincos_k(th, tk, &rr.sth, &rr.cth);
  const double sth = rr.sth, cth = rr.cth;
  const double arg = fma(m, cth, phi);
  const double acth = -a * cth, amsth = (a * m) * sth;
  if constexpr (SPLIT) ekf_sincos_row(arg, tk, rc, odd, rr.sa, rr.ca);
  else dfmi_sincos_k(arg, tk, &rr.sa, &rr.ca);
  const double sa = rr.sa, ca = rr.ca;
  const double h = fma(a, ca, dc);
  const double H[5] = {ca, acth * sa, -a * sa, amsth * sa, 1.0};
  const double y = xk - h;
  // (H P)_j from this lane's column (symmetric P): the chain of ekf_step
  const double hpj = fma(H[3], Pc[3], fma(H[2], Pc[2], fma(H[1], Pc[1], fma(H[0], Pc[0], Pc[4]))));
  double (&HP)[5] = rr.HP;
  HP[0] = row_bcast64<0>(HP[0], hpj);
  HP[1] = row_bcast64<1>(HP[1], hpj);
  HP[2] = row_bcast64<2>(HP[2], hpj);
  HP[3] = row_bcast64<3>(HP[3], hpj);
  HP[4] = row_bcast64<4>(HP[4], hpj);
  const double S = fma(HP[3], H[3], fma(HP[2], H[2], fma(HP[1], H[1], fma(HP[0], H[0], HP[4] + Rv))));
  double invS = __builtin_amdgcn_rcp(S);
  invS = fma(invS, fma(-S, invS, 1.0), invS);
  const double iy = invS * y;
  const double cj = hpj * invS;  // K_j
#pragma unroll
  for (int i = 0; i < 5; ++i) st[i] = fma(HP[i], iy, st[i]);
#pragma unroll
  for (int i = 0; i < 5; ++i) Pc[i] = fma(-HP[i], cj, Pc[i]);
}

// Same arguments and outputs as ekf_kernel; grid of ceil(nrec / 4) one-wave blocks.
// SPLIT: see ekf_row_step.
template <bool SPLIT>
__global__ __launch_bounds__(64) void ekf_row_kernel(const double* __restrict__ x, int64_t nrec, int64_t rec_stride,
                                                      int64_t n_samp, const double* __restrict__ x0,
                                                      const double* __restrict__ p0, const double* __restrict__ qd,
                                                      const double* __restrict__ rv, const double* __restrict__ wt,
                                                      int R, int64_t nbuf, double* __restrict__ states,
                                                      DfmiTrigK tk,
    const int* __restrict__ idx) {
  const int lane = threadIdx.x & 63;
  const int64_t r0 = (int64_t)blockIdx.x * 4 + (lane >> 4);
  const bool live = r0 < nrec;
  const int64_t r = live ? r0 : nrec - 1;  // rows past the end shadow the last channel (no stores)
  int j = lane & 15;
  if (j > 4) j = 4;
  // idx (optional): channel r of this launch is record idx[r] of the caller's arrays
  const int64_t rid = idx ? (int64_t)idx[r] : r;
  const double* __restrict__ xr = x + rid * rec_stride;
  double st[5], Pc[5], qv[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    st[i] = x0[rid * 5 + i];
    Pc[i] = (i == j) ? p0[i] : 0.0;
    qv[i] = (i == j) ? qd[i] : 0.0;
  }
  const double Rv = rv[rid];
  const bool writer = live && (lane & 15) == 0;
  int64_t to_snap = R;
  auto snap = [&](int64_t k) {
    if (--to_snap == 0) {
      to_snap = R;
      const int64_t b = (k + 1) / R - 1;
      if (b < nbuf && writer) {
#pragma unroll
        for (int i = 0; i < 5; ++i) states[(rid * nbuf + b) * 5 + i] = st[i];
      }
    }
  };
  constexpr int W = 1;  // table doubles per sample
  const bool odd = lane & 1;
  const RowSplitCoef rc = row_split_coef(tk, odd);
  RowRegs rr;
#pragma unroll
  for (int i = 0; i < 5; ++i) rr.HP[i] = 0.0;
  rr.sth = rr.cth = rr.sa = rr.ca = 0.0;
  auto step = [&](double xk, const double* w) { ekf_row_step<SPLIT>(st, Pc, qv, Rv, xk, w[0], tk, rr, rc, odd); };
  int64_t k = 0;
  double xc[8], wc[8][W];
  const int64_t n8 = n_samp & ~(int64_t)7;
  if (n8 > 0) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xc[u] = xr[u];
#pragma unroll
      for (int v = 0; v < W; ++v) wc[u][v] = wt[u * W + v];
    }
  }
  for (; k < n8; k += 8) {
    double xn[8], wn[8][W];
    // the next group, unconditionally (clamped into the record: no branch per load)
    const int64_t kn = k + 8 < n8 ? k + 8 : k;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xn[u] = xr[kn + u];
#pragma unroll
      for (int v = 0; v < W; ++v) wn[u][v] = wt[(kn + u) * W + v];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      step(xc[u], wc[u]);
      snap(k + u);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xc[u] = xn[u];
#pragma unroll
      for (int v = 0; v < W; ++v) wc[u][v] = wn[u][v];
    }
  }
  for (; k < n_samp; ++k) {
    step(xr[k], wt + k * W);
    snap(k);
  }
}

// ---------------------------------------------------------------------------
// Row kernel with sincos by ROTATION (round 3, the default for few channels when R % 4 == 0).
// Both sincos arguments move little from one sample to the next: theta_k - theta_{k-1} is
// w_m / f_samp plus the change of psi (0.031 rad at config 5), phi + m cos(theta) moves by
// at most ~m w_m / f_samp. The row evaluates the full Cody-Waite sincos (ekf_sincos_row) on
// the first sample of every group of G = 16 (8 or 4 when R is not a multiple of 16), the
// anchor, and on the
// others rotates the previous sample's (sin, cos) by d = x_k - x_{k-1}:
//   sin x_k = sin x_{k-1} cos d + cos x_{k-1} sin d,  cos x_k = cos x_{k-1} cos d - sin x_{k-1} sin d,
// with sin d / cos d from the same kernel coefficients (|d| < 0.78: no reduction, no quadrant).
// The argument is the reference's: x_k is formed exactly as before (fl(w_m t_k + psi),
// fl(phi + m cos theta)) and d is the difference of two such doubles (exact when they lie
// within a factor 2 of each other, else off by half an ulp of d), so sin / cos are of the
// same rounded argument; only the rotation's rounding (~1 ulp per step, reset at every
// anchor) differs from the anchor form. Per sincos this replaces the reduction, the
// quadrant selects and the library-range test (~38 instructions with the lane split) by
// ~17 (d, the one-polynomial pair, 2 DPP moves, 4 for the rotation): ~89 (G = 8) / ~85
// (G = 16) instead of ~123 wave instructions per sample; config 5 3.74 -> 5.62 (G = 8) ->
// 5.83 M samples/s per channel (profiles/r03s_ekf_rot_ab.jsonl, r03s_ekf_rot_g_newton_ab.json).
// A group in which any |d| reaches 0.78 (fast modulation, a diverging state) is rolled
// back and re-run with the anchor form on every sample (per row: a channel's result never
// depends on another channel's data). Snapshots fall on group ends (R % G == 0, checked by
// the host), so the per-sample snapshot countdown is per group here.
// ---------------------------------------------------------------------------

// sin d / cos d for |d| < 0.78 on a row with dfmi_sincos_k's kernel coefficients, written as
// one degree-7 polynomial in z = d^2 per lane: even lanes sin d = d (1 + z P_s(z)), odd lanes
// cos d = 1 + z (-1/2 + z P_c(z)), i.e. v = mult * Poly(z) with mult = d on even lanes and 1
// on odd ones (mult = fma(e, d, 1 - e), exact); read back by DPP into the tied registers
// sn / cs. 12 instructions for the pair (no reduction, no quadrant, no selects).
struct RotCoef {
  double c[8];   // z^7 .. z^0
  double e, e1;  // 1, 0 on even lanes; 0, 1 on odd lanes
};
__device__ __forceinline__ RotCoef rot_coef(const DfmiTrigK& k, int par) {
  RotCoef rc;
  if (par) {
#pragma unroll
    for (int i = 0; i < 6; ++i) rc.c[i] = k.c[10 + i];
    rc.c[6] = -0.5;
  } else {
    rc.c[0] = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) rc.c[1 + i] = k.c[4 + i];
  }
  rc.c[7] = 1.0;
  rc.e = par ? 0.0 : 1.0;
  rc.e1 = par ? 1.0 : 0.0;
  return rc;
}
__device__ __forceinline__ void ekf_sincos_row_small(double d, const RotCoef& rc, double& sn, double& cs) {
  const double z = d * d;
  double p = fma(z, rc.c[0], rc.c[1]);
#pragma unroll
  for (int i = 2; i < 8; ++i) p = fma(z, p, rc.c[i]);
  const double v = fma(rc.e, d, rc.e1) * p;
  sn = row_bcast64<0>(sn, v);
  cs = row_bcast64<1>(cs, v);
}

#ifndef DFMI_EKF_ROT_NEWTON
#define DFMI_EKF_ROT_NEWTON 1  // 1/S: v_rcp_f64 + one Newton step (without: +6 % but 2.7e-12 from the C oracle, r03s)
#endif
#ifndef DFMI_EKF_ROT_G
#define DFMI_EKF_ROT_G 16  // samples per anchor where R % G == 0 (8 measured 4 % slower, r03s; A/B builds)
#endif

struct RotRegs {
  double HP[5];
  double sth, cth, sa, ca;  // sincos of the previous sample's theta / phase argument (the rotation bases)
  double thp, argp;         // the previous sample's theta / phase argument
  double sd, cd;            // DPP destinations of sin d / cos d
};

// One sample. ROT = false: anchor (full sincos); true: rotation of the bases by d, |d| folded
// into dmax.
template <bool ROT>
__device__ __forceinline__ void ekf_rot_step(double (&st)[5], double (&Pc)[5], const double (&qv)[5], double Rv,
                                             double xk, double wt, const DfmiTrigK& tk, RotRegs& rr,
                                             const RowSplitCoef& rc, const RotCoef& ro, bool odd, double& dmax) {
#pragma unroll
  for (int i = 0; i < 5; ++i) Pc[i] = Pc[i] + qv[i];
  const double a = st[0], m = st[1], phi = st[2], psi = st[3], dc = st[4];
  const double th = wt + psi;
  if constexpr (ROT) {
    const double d = th - rr.thp;
    dmax = fmax(dmax, fabs(d));
    ekf_sincos_row_small(d, ro, rr.sd, rr.cd);
    const double s = fma(rr.sth, rr.cd, rr.cth * rr.sd);
    const double c = fma(rr.cth, rr.cd, -(rr.sth * rr.sd));
    rr.sth = s;
    rr.cth = c;
  } else {
    ekf_sincos_row(th, tk, rc, odd, rr.sth, rr.cth);
  }
  rr.thp = th;
  const double sth = rr.sth, cth = rr.cth;
  const double arg = fma(m, cth, phi);
  const double acth = -a * cth, amsth = (a * m) * sth;
  if constexpr (ROT) {
    const double d = arg - rr.argp;
    dmax = fmax(dmax, fabs(d));
    ekf_sincos_row_small(d, ro, rr.sd, rr.cd);
    const double s = fma(rr.sa, rr.cd, rr.ca * rr.sd);
    const double c = fma(rr.ca, rr.cd, -(rr.sa * rr.sd));
    rr.sa = s;
    rr.ca = c;
  } else {
    ekf_sincos_row(arg, tk, rc, odd, rr.sa, rr.ca);
  }
  rr.argp = arg;
  const double sa = rr.sa, ca = rr.ca;
  const double h = fma(a, ca, dc);
  const double H[5] = {ca, acth * sa, -a * sa, amsth * sa, 1.0};
  const double y = xk - h;
  const double hpj = fma(H[3], Pc[3], fma(H[2], Pc[2], fma(H[1], Pc[1], fma(H[0], Pc[0], Pc[4]))));
  double (&HP)[5] = rr.HP;
  HP[0] = row_bcast64<0>(HP[0], hpj);
  HP[1] = row_bcast64<1>(HP[1], hpj);
  HP[2] = row_bcast64<2>(HP[2], hpj);
  HP[3] = row_bcast64<3>(HP[3], hpj);
  HP[4] = row_bcast64<4>(HP[4], hpj);
  const double S = fma(HP[3], H[3], fma(HP[2], H[2], fma(HP[1], H[1], fma(HP[0], H[0], HP[4] + Rv))));
  double invS = __builtin_amdgcn_rcp(S);
#if DFMI_EKF_ROT_NEWTON
  invS = fma(invS, fma(-S, invS, 1.0), invS);
#endif
  const double iy = invS * y;
  const double cj = hpj * invS;
#pragma unroll
  for (int i = 0; i < 5; ++i) st[i] = fma(HP[i], iy, st[i]);
#pragma unroll
  for (int i = 0; i < 5; ++i) Pc[i] = fma(-HP[i], cj, Pc[i]);
}

// Same arguments, grid and outputs as ekf_row_kernel; R % G == 0 (host-checked).
template <int G>
__global__ __launch_bounds__(64) void ekf_rot_kernel(const double* __restrict__ x, int64_t nrec, int64_t rec_stride,
                                                      int64_t n_samp, const double* __restrict__ x0,
                                                      const double* __restrict__ p0, const double* __restrict__ qd,
                                                      const double* __restrict__ rv, const double* __restrict__ wt,
                                                      int R, int64_t nbuf, double* __restrict__ states,
                                                      DfmiTrigK tk,
    const int* __restrict__ idx) {
  const int lane = threadIdx.x & 63;
  const int64_t r0 = (int64_t)blockIdx.x * 4 + (lane >> 4);
  const bool live = r0 < nrec;
  const int64_t r = live ? r0 : nrec - 1;
  int j = lane & 15;
  if (j > 4) j = 4;
  // idx (optional): channel r of this launch is record idx[r] of the caller's arrays
  const int64_t rid = idx ? (int64_t)idx[r] : r;
  const double* __restrict__ xr = x + rid * rec_stride;
  double st[5], Pc[5], qv[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    st[i] = x0[rid * 5 + i];
    Pc[i] = (i == j) ? p0[i] : 0.0;
    qv[i] = (i == j) ? qd[i] : 0.0;
  }
  const double Rv = rv[rid];
  const bool writer = live && (lane & 15) == 0;
  const bool odd = lane & 1;
  const RowSplitCoef rc = row_split_coef(tk, odd);
  const RotCoef ro = rot_coef(tk, odd);
  RotRegs rr;
#pragma unroll
  for (int i = 0; i < 5; ++i) rr.HP[i] = 0.0;
  rr.sth = rr.cth = rr.sa = rr.ca = rr.thp = rr.argp = rr.sd = rr.cd = 0.0;
  double dmax = 0.0;
  int64_t k = 0;
  const int64_t ng = n_samp / G;
  int64_t to_snap = R;
  double xc[G], wc[G];
  if (ng > 0) {
#pragma unroll
    for (int u = 0; u < G; ++u) {
      xc[u] = xr[u];
      wc[u] = wt[u];
    }
  }
  for (int64_t g = 0; g < ng; ++g, k += G) {
    double xn[G], wn[G];
    const int64_t kn = g + 1 < ng ? k + G : k;
#pragma unroll
    for (int u = 0; u < G; ++u) {
      xn[u] = xr[kn + u];
      wn[u] = wt[kn + u];
    }
    double st0[5], Pc0[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      st0[i] = st[i];
      Pc0[i] = Pc[i];
    }
    dmax = 0.0;
    ekf_rot_step<false>(st, Pc, qv, Rv, xc[0], wc[0], tk, rr, rc, ro, odd, dmax);
#pragma unroll
    for (int u = 1; u < G; ++u) ekf_rot_step<true>(st, Pc, qv, Rv, xc[u], wc[u], tk, rr, rc, ro, odd, dmax);
    if (__builtin_expect(dmax >= 0.78, 0)) {  // this row: redo the group with the anchor form throughout
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        st[i] = st0[i];
        Pc[i] = Pc0[i];
      }
#pragma unroll
      for (int u = 0; u < G; ++u) ekf_rot_step<false>(st, Pc, qv, Rv, xc[u], wc[u], tk, rr, rc, ro, odd, dmax);
    }
    to_snap -= G;
    if (to_snap == 0) {
      to_snap = R;
      const int64_t b = (k + G) / R - 1;
      if (b < nbuf && writer) {
#pragma unroll
        for (int i = 0; i < 5; ++i) states[(rid * nbuf + b) * 5 + i] = st[i];
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      xc[u] = xn[u];
      wc[u] = wn[u];
    }
  }
  // the last n_samp % G samples (no snapshot can fall here: R is a multiple of G)
  for (; k < n_samp; ++k) ekf_rot_step<false>(st, Pc, qv, Rv, xr[k], wt[k], tk, rr, rc, ro, odd, dmax);
}

// ---------------------------------------------------------------------------
// Lane kernel (many channels: lane = channel) with the same anchored rotation as
// ekf_rot_kernel: sin / cos of d by both kernel polynomials in the lane (no row to split
// them over), the anchor and the fallback group (any |d| >= 0.78, per lane) by
// dfmi_sincos_k; otherwise ekf_step's expressions. ~2 x 20 instructions per sample fewer
// than ekf_kernel's two full sincos.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ekf_rotate_lane(double d, const DfmiTrigK& k, double& s, double& c) {
  const double z = d * d;
  const double ps = fma(z, fma(z, fma(z, fma(z, fma(z, k.c[4], k.c[5]), k.c[6]), k.c[7]), k.c[8]), k.c[9]);
  const double sd = fma(d * z, ps, d);
  const double pc = fma(z, fma(z, fma(z, fma(z, fma(z, k.c[10], k.c[11]), k.c[12]), k.c[13]), k.c[14]), k.c[15]);
  const double cd = fma(z * z, pc, fma(-0.5, z, 1.0));
  const double sn = fma(s, cd, c * sd);
  c = fma(c, cd, -(s * sd));
  s = sn;
}

struct LaneRot {
  double sth, cth, sa, ca, thp, argp;
};

template <bool ROT>
__device__ __forceinline__ void ekf_step_rot(double (&st)[5], double (&P)[5][5], const double (&Q)[5], double Rv,
                                             double xk, double wt, const DfmiTrigK& tk, LaneRot& lr, double& dmax) {
#pragma unroll
  for (int i = 0; i < 5; ++i) P[i][i] = P[i][i] + Q[i];
  const double a = st[0], m = st[1], phi = st[2], psi = st[3], dc = st[4];
  const double th = wt + psi;
  if constexpr (ROT) {
    const double d = th - lr.thp;
    dmax = fmax(dmax, fabs(d));
    ekf_rotate_lane(d, tk, lr.sth, lr.cth);
  } else {
    dfmi_sincos_k(th, tk, &lr.sth, &lr.cth);
  }
  lr.thp = th;
  const double sth = lr.sth, cth = lr.cth;
  const double arg = fma(m, cth, phi);
  const double acth = -a * cth, amsth = (a * m) * sth;
  if constexpr (ROT) {
    const double d = arg - lr.argp;
    dmax = fmax(dmax, fabs(d));
    ekf_rotate_lane(d, tk, lr.sa, lr.ca);
  } else {
    dfmi_sincos_k(arg, tk, &lr.sa, &lr.ca);
  }
  lr.argp = arg;
  const double sa = lr.sa, ca = lr.ca;
  const double h = fma(a, ca, dc);
  const double H[5] = {ca, acth * sa, -a * sa, amsth * sa, 1.0};
  const double y = xk - h;
  auto Pu = [&](int i, int j) -> double { return i <= j ? P[i][j] : P[j][i]; };
  double HP[5];
#pragma unroll
  for (int j = 0; j < 5; ++j)
    HP[j] = fma(H[3], Pu(3, j), fma(H[2], Pu(2, j), fma(H[1], Pu(1, j), fma(H[0], Pu(0, j), Pu(4, j)))));
  const double S = fma(HP[3], H[3], fma(HP[2], H[2], fma(HP[1], H[1], fma(HP[0], H[0], HP[4] + Rv))));
  double invS = __builtin_amdgcn_rcp(S);
  invS = fma(invS, fma(-S, invS, 1.0), invS);
  const double iy = invS * y;
  double K[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) K[i] = HP[i] * invS;
#pragma unroll
  for (int i = 0; i < 5; ++i) st[i] = fma(HP[i], iy, st[i]);
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j)
      if (j >= i) P[i][j] = fma(-K[i], HP[j], P[i][j]);
}

// Same arguments, grid and outputs as ekf_kernel; R % G == 0 (host-checked).
template <int G>
__global__ __launch_bounds__(64) void ekf_lane_rot_kernel(const double* __restrict__ x, int64_t nrec,
                                                           int64_t rec_stride, int64_t n_samp,
                                                           const double* __restrict__ x0, const double* __restrict__ p0,
                                                           const double* __restrict__ qd, const double* __restrict__ rv,
                                                           const double* __restrict__ wt, int R, int64_t nbuf,
                                                           double* __restrict__ states, DfmiTrigK tk,
    const int* __restrict__ idx) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrec) return;
  // idx (optional): channel r of this launch is record idx[r] of the caller's arrays
  const int64_t rid = idx ? (int64_t)idx[r] : r;
  const double* __restrict__ xr = x + rid * rec_stride;
  double st[5], P[5][5], Q[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    st[i] = x0[rid * 5 + i];
    Q[i] = qd[i];
#pragma unroll
    for (int j = 0; j < 5; ++j) P[i][j] = (i == j) ? p0[i] : 0.0;
  }
  const double Rv = rv[rid];
  LaneRot lr{0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  double dmax = 0.0;
  int64_t k = 0;
  const int64_t ng = n_samp / G;
  int64_t to_snap = R;
  double xc[G], wc[G];
  if (ng > 0) {
#pragma unroll
    for (int u = 0; u < G; ++u) {
      xc[u] = xr[u];
      wc[u] = wt[u];
    }
  }
  for (int64_t g = 0; g < ng; ++g, k += G) {
    double xn[G], wn[G];
    const int64_t kn = g + 1 < ng ? k + G : k;
#pragma unroll
    for (int u = 0; u < G; ++u) {
      xn[u] = xr[kn + u];
      wn[u] = wt[kn + u];
    }
    double st0[5], P0[5][5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      st0[i] = st[i];
#pragma unroll
      for (int j = 0; j < 5; ++j)
        if (j >= i) P0[i][j] = P[i][j];
    }
    dmax = 0.0;
    ekf_step_rot<false>(st, P, Q, Rv, xc[0], wc[0], tk, lr, dmax);
#pragma unroll
    for (int u = 1; u < G; ++u) ekf_step_rot<true>(st, P, Q, Rv, xc[u], wc[u], tk, lr, dmax);
    if (__builtin_expect(dmax >= 0.78, 0)) {  // this lane: redo the group with the anchor form throughout
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        st[i] = st0[i];
#pragma unroll
        for (int j = 0; j < 5; ++j)
          if (j >= i) P[i][j] = P0[i][j];
      }
#pragma unroll
      for (int u = 0; u < G; ++u) ekf_step_rot<false>(st, P, Q, Rv, xc[u], wc[u], tk, lr, dmax);
    }
    to_snap -= G;
    if (to_snap == 0) {
      to_snap = R;
      const int64_t b = (k + G) / R - 1;
      if (b < nbuf) {
#pragma unroll
        for (int i = 0; i < 5; ++i) states[(rid * nbuf + b) * 5 + i] = st[i];
      }
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
      xc[u] = xn[u];
      wc[u] = wn[u];
    }
  }
  for (; k < n_samp; ++k) ekf_step_rot<false>(st, P, Q, Rv, xr[k], wt[k], tk, lr, dmax);
}

}  // namespace dfmi
