// ekf_pit.h — the EKF of fitters.py:214-320 parallel in time (the default for up to 1,024
// channels of >= 4,096 samples; the block size grows with the channel count, ekf_pit_run).
//
// The sequential kernels (ekf.h) run one channel's samples in order: ~410 clocks per
// sample on one SIMD, a floor of the dependent fp64 chain (DESIGN.md §4, r04c PMC), so a
// single 400k-sample channel takes ~69 ms however large the GPU is. Here the channel is cut
// into nb blocks of B samples and the filter is solved as a fixed point:
//
//   1. linearize the measurement h(x) = a cos(phi + m cos(w_m t_k + psi)) + dc at a
//      trajectory xbar_k (predicted states; on the first pass the head's sequential EKF over
//      the first 256 samples, then the state entering sample 256), so the model is
//      linear-Gaussian: x_k = x_{k-1} + q, y_k = H_k x_k + d_k + r (F = I as in the reference);
//   2. the linear Kalman filter of that model is an associative prefix scan over filtering
//      elements (A, b, C, eta, J) (Sarkka & Garcia-Fernandez, "Temporal parallelization of
//      Bayesian smoothers", IEEE TAC 2021): every block folds its B elements in order (a
//      rank-1 form of the combine per sample), the block aggregates are scanned
//      (ekf_pit_scan_kernel: Hillis-Steele in LDS, 64 per workgroup, four waves per combine,
//      over a hierarchy of workgroup totals made true prefixes top-down by
//      ekf_pit_fixup_kernel), and the inclusive prefix at block b-1 is the filtered (mean,
//      covariance) entering block b;
//   3. each block then runs the TRUE EKF (ekf_step, the lane kernel's arithmetic) from that
//      entry state, which gives the snapshots and the next trajectory. ekf_pit_pass_kernel
//      does 3 and the next pass's fold of 2 in one sweep: the element of a sample is
//      linearized at the state entering it, which is the EKF step's own predicted state (its H
//      and h(x) are already formed). The first pass's aggregates come from
//      ekf_pit_aggregate_kernel at the seeded trajectory (ekf_pit_head_kernel); the separate
//      aggregate / ekf_pit_blocks_kernel pair per pass remains behind the ekf_pit_fused knob.
//
// Convergence (pit_decide, on the device: the pass kernel's last workgroup of a channel, or
// ekf_pit_check_kernel on the unfused path) bounds the distance of the output snapshots from
// the iteration's fixed point by rho / (1 - rho) d_k <= 1e-13, with d_k their largest relative
// move in pass k and rho the contraction measured per channel; the fixed point is the EKF
// itself to the scan's rounding, so the output is the sequential EKF's to rounding. A
// converged channel's later kernels return at once (status per channel); the host reads the
// count of channels still passing after the first ekf_pit_first passes and then every
// ekf_pit_every, and stops when none is left. A channel that stops contracting (or reaches
// the pass cap) is re-run by the sequential row / lane kernel reading the record in place
// (ekf_pit_handover_kernel's index list; after the passes by default, ekf_pit_overlap in
// dfmi_capi.hip), so the result never depends on the iteration having converged.
//
// Layouts (all channel-major, blocks fastest so lane b of a wave reads address b):
//   xt[r][i][b], wtt[i][b] (sample k = b B + i), xbar[r][c][i][b] (the seeded trajectory:
//   the unfused path only; the fused first pass reads the head's states directly),
//   scan level l: [r][65][n_l] with n_0 = nb, n_{l+1} = ceil(n_l / 64), two buffers (a pass
//   reads one and writes the other), ent[r][c][b] (the previous pass's entry states).
// Element components: A 0..24 (row-major), b 25..29, C 30..44 (upper triangle, row-major),
// eta 45..49, J 50..64 (upper triangle).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "dfmi_math.h"
#include "ekf.h"

namespace dfmi {

constexpr int kPitEl = 65;
constexpr int kPitA = 0, kPitB = 25, kPitC = 30, kPitE = 45, kPitJ = 50;
constexpr int kPitWg = 64;  // elements per scan workgroup (every level of the scan hierarchy)
__host__ __device__ constexpr int pit_sy(int i, int j) {
  return i <= j ? i * 5 - i * (i - 1) / 2 + (j - i) : j * 5 - j * (j - 1) / 2 + (i - j);
}
__host__ __device__ constexpr double pit_identity(int c) {
  return (c < kPitB && c / 5 == c % 5) ? 1.0 : 0.0;  // A = I, everything else 0
}

// Per-channel control of the passes (device, 64 B). status: 0 passing, 1 converged, 2 not
// contracting (the host re-runs it with the sequential kernel); every pass kernel of a channel
// whose status is set returns at once.
constexpr int kPitTrend = 4;  // passes over which the stall test measures the contraction
struct PitChan {
  int status;
  int passes;  // passes run
  int stall;   // consecutive passes that did not contract fast enough (pit_decide)
  int pad;
  double dprev;              // the previous pass's move d (NaN before the second pass)
  double rho;                // the last trusted contraction d_k / d_{k-1} (-1: none yet)
  double dold[kPitTrend];    // moves of the passes k-1 .. k-kPitTrend (NaN: none)
};

// The stop rule (round 5). d_k = the largest relative move, max |x_k - x_{k-1}| / max(1, |x_k|),
// of the channel's OUTPUT snapshots (fitters.py:305-307) between passes k-1 and k (measure 0;
// measure 1, diagnostics: the block-entry states, whose rounding noise after the scan reached
// 1e-12 on a stiff filter, profiles/r05a). For a fixed-point iteration contracting by rho per
// pass, the distance of x_k from the fixed point is at most rho / (1 - rho) d_k; the channel
// is converged when that bound is <= tol (1e-13), rho estimated on the device from the moves
// (the larger of the last two ratios d_k / d_{k-1}). Ratios of moves at or below the rounding
// noise (`noise` = tol) say nothing about the contraction, so there the last trusted ratio
// stands in. A pass over which the channel does not contract (the geometric-mean contraction
// of the last 4 passes >= 1), or contracts too slowly to meet the bound within the cap (>= 0.5
// and the passes it would still need push it past the cap), counts towards `stall`; stall_max
// such passes in a row, or a non-finite move after the first pass (the filter's own states are
// not finite), hand the channel to the sequential kernel, as does the host's cap
// (ekf_pit_passes). A pass costs ~1/1000 of the sequential kernel on one
// 400k-sample channel, so the passes go on as long as the bound can still be met.
struct PitRule {
  double tol;
  double noise;      // moves at or below this are rounding: their ratios are not trusted
  int stall_max;
  int cap;           // the host's pass cap (ekf_pit_passes)
  int slow_from;     // passes before the too-slow-for-the-cap test applies (ekf_pit_slow_from, 16)
  int hist_n;        // moves recorded per channel into hist (0: none)
  int measure;       // 0: the output snapshots' move (default); 1: the block-entry states' move
};

// A snapshot (fitters.py:305-307) written by this pass: its largest relative move since the
// previous pass's value at the same place (the states buffer itself: zeros before the first
// pass, whose move pit_decide ignores) into d.
__host__ __device__ __forceinline__ void pit_snapshot(double* __restrict__ so, const double (&st)[5], double& d) {
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    const double m = fabs(st[c] - so[c]) / fmax(1.0, fabs(st[c]));
    d = m <= d ? d : m;  // NaN propagates
    so[c] = st[c];
  }
}

__host__ __device__ __forceinline__ void pit_decide(PitChan& c, double d, const PitRule& ru, double* hist) {
  const int pass = c.passes;
  c.passes = pass + 1;
  if (pass == 0) d = __builtin_nan("");  // no previous pass to have moved from
  if (hist && pass < ru.hist_n) hist[pass] = d;
  int status = 0;
  const double dprev = c.dprev;
  if (d == 0.0) {
    status = 1;  // nothing moved at all: the fixed point itself
  } else if (!(d <= 1.7976931348623157e308)) {
    if (pass >= 1) status = 2;  // the filter's own states are not finite: the sequential kernel
  } else {
    // rho: the contraction of this pass, trusted when both moves stand above the rounding
    // noise; the bound uses the larger of the last two trusted ratios (one move that happens
    // to be small, e.g. a snapshot crossing its old value, does not end the passes)
    double rho = -1.0;
    if (dprev > 0.0 && dprev <= 1.7976931348623157e308) {
      const double q = d / dprev;
      if (dprev > ru.noise && d > ru.noise) {
        rho = c.rho >= 0.0 ? fmax(q, c.rho) : q;
        c.rho = q;
      } else if (d > ru.noise) {
        rho = q;  // out of the noise again: a real move
      } else {
        rho = c.rho;  // at the noise: the last trusted contraction stands
      }
    }
    if (rho < 0.0) {
      if (d <= ru.noise) status = 1;  // no ratio yet, the move itself at the rounding noise
    } else if (rho < 1.0 && rho / (1.0 - rho) * d <= ru.tol) {
      status = 1;
    }
    // moves that alternate large / small (a period-2 component of the iteration: single-pass
    // ratios above and below 1 while every second pass contracts) never meet the bound above;
    // their envelope D_k = max(d_k, d_{k-1}) decays by r = (D_k / D_{k-2})^(1/2) per pass and
    // bounds the distance from the fixed point by 2 D_k r / (1 - r) (round 6: 9 of the stress
    // set's well-conditioned channels ran into the cap this way, profiles/r06/ekf_pit_rule_replay.txt)
    if (status == 0 && pass >= 3) {
      const double dk = fmax(d, c.dold[0]), dk2 = fmax(c.dold[1], c.dold[2]);
      if (dk > 0.0 && dk <= 1.7976931348623157e308 && dk2 > 0.0 && dk2 <= 1.7976931348623157e308) {
        const double r = sqrt(dk / dk2);
        if (r < 1.0 && 2.0 * dk * r / (1.0 - r) <= ru.tol) status = 1;
      }
    }
    if (status == 0 && d > ru.noise) {
      // not contracting, or too slowly to meet the bound within the cap: stall_max passes in
      // a row of that hand the channel to the sequential kernel. The contraction here is the
      // geometric mean over the last kPitTrend passes (a crawling start-up transient
      // alternates good and bad single ratios)
      int w = 0;
      double dw = 0.0;
#pragma unroll
      for (int i = 0; i < kPitTrend; ++i)
        if (c.dold[i] > 0.0 && c.dold[i] <= 1.7976931348623157e308) {
          w = i + 1;
          dw = c.dold[i];
        }
      if (w > 0) {
        const double rt = pow(d / dw, 1.0 / w);
        bool slow = rt >= 1.0;
        // the extrapolation to the cap only after the start-up transient: the contraction of
        // these iterations improves as the trajectory nears the fixed point, and judged at pass
        // 5 it handed 42 well-conditioned stress channels (that converged by pass 43) over
        if (!slow && rt >= 0.5 && pass + 1 >= ru.slow_from) {
          const double need = log(ru.tol * (1.0 - rt) / (rt * d)) / log(rt);
          slow = pass + 1 + need > ru.cap;
        }
        c.stall = slow ? c.stall + 1 : 0;
        if (c.stall >= ru.stall_max) status = 2;
      }
    }
  }
#pragma unroll
  for (int i = kPitTrend - 1; i > 0; --i) c.dold[i] = c.dold[i - 1];
  c.dold[0] = d;
  c.dprev = d;
  c.status = status;
}

// a filtering element read through a strided pointer (global SoA or LDS)
struct PitEl {
  const double* p;
  int64_t ld;
  __device__ __forceinline__ double operator()(int c) const { return p[c * ld]; }
  __device__ __forceinline__ double A(int r, int c) const { return p[(kPitA + r * 5 + c) * ld]; }
  __device__ __forceinline__ double C(int i, int j) const { return p[(kPitC + pit_sy(i, j)) * ld]; }
  __device__ __forceinline__ double J(int i, int j) const { return p[(kPitJ + pit_sy(i, j)) * ld]; }
};

// o = ei (x) ej, ei the earlier element (Sarkka & Garcia-Fernandez, Lemma 8):
//   M = (I + C_i J_j)^-1, A = A_j M A_i, b = A_j M (b_i + C_i eta_j) + b_j,
//   C = A_j M C_i A_j^T + C_j, eta = A_i^T M^T (eta_j - J_j b_i) + eta_i,
//   J = A_i^T M^T J_j A_i + J_i.
// M by Gauss-Jordan (I + C J with C, J PSD has eigenvalues >= 1 but its leading minors can
// vanish: a pivot below 1/4 redoes it with partial pivoting, whose row swaps are selects so
// every index stays static).
__device__ __forceinline__ void pit_minv(const PitEl& ei, const PitEl& ej, double (&M)[5][5]) {
  double T[5][10];
  auto init_T = [&]() {
#pragma unroll
    for (int r = 0; r < 5; ++r) {
#pragma unroll
      for (int c = 0; c < 5; ++c) {
        double s = (r == c) ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < 5; ++k) s = fma(ei.C(r, k), ej.J(k, c), s);
        T[r][c] = s;
        T[r][5 + c] = (r == c) ? 1.0 : 0.0;
      }
    }
  };
  init_T();
  // without pivoting first (T = I + C J is I plus a small term for every element the passes
  // meet: pivots near 1); any pivot below 1/4 in magnitude redoes it with partial pivoting
  double pmin = 1.0;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    pmin = fmin(pmin, fabs(T[k][k]));
    const double ip = 1.0 / T[k][k];
#pragma unroll
    for (int c = k + 1; c < 10; ++c) T[k][c] *= ip;
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      if (r == k) continue;
      const double f = T[r][k];
#pragma unroll
      for (int c = k + 1; c < 10; ++c) T[r][c] = fma(-f, T[k][c], T[r][c]);
    }
  }
  if (__builtin_expect(!(pmin >= 0.25), 0)) {
    init_T();
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      int p = k;
      double best = fabs(T[k][k]);
#pragma unroll
      for (int r = k + 1; r < 5; ++r) {
        const double v = fabs(T[r][k]);
        if (v > best) {
          best = v;
          p = r;
        }
      }
#pragma unroll
      for (int r = k + 1; r < 5; ++r) {
        const bool sw = p == r;
#pragma unroll
        for (int c = k; c < 10; ++c) {
          const double t = T[k][c];
          T[k][c] = sw ? T[r][c] : t;
          T[r][c] = sw ? t : T[r][c];
        }
      }
      const double ip = 1.0 / T[k][k];
#pragma unroll
      for (int c = k + 1; c < 10; ++c) T[k][c] *= ip;
#pragma unroll
      for (int r = 0; r < 5; ++r) {
        if (r == k) continue;
        const double f = T[r][k];
#pragma unroll
        for (int c = k + 1; c < 10; ++c) T[r][c] = fma(-f, T[k][c], T[r][c]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 5; ++r)
#pragma unroll
    for (int c = 0; c < 5; ++c) M[r][c] = T[r][5 + c];
}

// The combine split in four roles with no shared intermediate beyond M, so four waves can
// form one element's result side by side (ekf_pit_scan_kernel): role 0 A (25 outputs), role 1
// b and eta (10), role 2 C (15), role 3 J (15). pit_role_comp maps a role's output slot to
// the element component it holds.
template <int ROLE>
__host__ __device__ constexpr int pit_role_n() {
  return ROLE == 0 ? 25 : ROLE == 1 ? 10 : 15;
}
template <int ROLE>
__host__ __device__ constexpr int pit_role_comp(int i) {
  return ROLE == 0 ? kPitA + i : ROLE == 1 ? (i < 5 ? kPitB + i : kPitE + i - 5) : ROLE == 2 ? kPitC + i : kPitJ + i;
}
template <int ROLE>
__device__ __forceinline__ void pit_role(const PitEl& ei, const PitEl& ej, const double (&M)[5][5], double (&o)[25]) {
  if constexpr (ROLE == 0) {  // A = A_j (M A_i)
    double X[5][5];
#pragma unroll
    for (int r = 0; r < 5; ++r)
#pragma unroll
      for (int c = 0; c < 5; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 5; ++k) s = fma(M[r][k], ei.A(k, c), s);
        X[r][c] = s;
      }
#pragma unroll
    for (int r = 0; r < 5; ++r)
#pragma unroll
      for (int c = 0; c < 5; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 5; ++k) s = fma(ej.A(r, k), X[k][c], s);
        o[r * 5 + c] = s;
      }
  } else if constexpr (ROLE == 1) {  // b = A_j M (b_i + C_i eta_j) + b_j; eta = A_i^T M^T (eta_j - J_j b_i) + eta_i
    double w[5], mw[5], y[5], z[5];
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      double s = ei(kPitB + r);
#pragma unroll
      for (int k = 0; k < 5; ++k) s = fma(ei.C(r, k), ej(kPitE + k), s);
      w[r] = s;
      double t = ej(kPitE + r);
#pragma unroll
      for (int k = 0; k < 5; ++k) t = fma(-ej.J(r, k), ei(kPitB + k), t);
      y[r] = t;
    }
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      double s = 0.0, t = 0.0;
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        s = fma(M[r][k], w[k], s);
        t = fma(M[k][r], y[k], t);
      }
      mw[r] = s;
      z[r] = t;
    }
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      double s = ej(kPitB + r), t = ei(kPitE + r);
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        s = fma(ej.A(r, k), mw[k], s);
        t = fma(ei.A(k, r), z[k], t);
      }
      o[r] = s;
      o[5 + r] = t;
    }
  } else if constexpr (ROLE == 2) {  // C = A_j (M C_i) A_j^T + C_j, M C_i symmetric
    double X[5][5], Y[5][5];
#pragma unroll
    for (int r = 0; r < 5; ++r)
#pragma unroll
      for (int c = r; c < 5; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 5; ++k) s = fma(M[r][k], ei.C(k, c), s);
        X[r][c] = s;
        X[c][r] = s;
      }
#pragma unroll
    for (int r = 0; r < 5; ++r)
#pragma unroll
      for (int c = 0; c < 5; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 5; ++k) s = fma(X[r][k], ej.A(c, k), s);
        Y[r][c] = s;
      }
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = i; j < 5; ++j) {
        double s = ej.C(i, j);
#pragma unroll
        for (int k = 0; k < 5; ++k) s = fma(ej.A(i, k), Y[k][j], s);
        o[pit_sy(i, j)] = s;
      }
  } else {  // J = A_i^T (M^T J_j) A_i + J_i, M^T J_j symmetric
    double X[5][5], Y[5][5];
#pragma unroll
    for (int r = 0; r < 5; ++r)
#pragma unroll
      for (int c = r; c < 5; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 5; ++k) s = fma(M[k][r], ej.J(k, c), s);
        X[r][c] = s;
        X[c][r] = s;
      }
#pragma unroll
    for (int r = 0; r < 5; ++r)
#pragma unroll
      for (int c = 0; c < 5; ++c) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 5; ++k) s = fma(X[r][k], ei.A(k, c), s);
        Y[r][c] = s;
      }
#pragma unroll
    for (int i = 0; i < 5; ++i)
#pragma unroll
      for (int j = i; j < 5; ++j) {
        double s = ei.J(i, j);
#pragma unroll
        for (int k = 0; k < 5; ++k) s = fma(ei.A(k, i), Y[k][j], s);
        o[pit_sy(i, j)] = s;
      }
  }
}

template <int ROLE>
__device__ __forceinline__ void pit_role_into(const PitEl& ei, const PitEl& ej, const double (&M)[5][5],
                                              double (&o)[kPitEl]) {
  double t[25];
  pit_role<ROLE>(ei, ej, M, t);
#pragma unroll
  for (int i = 0; i < pit_role_n<ROLE>(); ++i) o[pit_role_comp<ROLE>(i)] = t[i];
}

// the whole combine in one lane
__device__ __forceinline__ void pit_combine(const PitEl& ei, const PitEl& ej, double (&o)[kPitEl]) {
  double M[5][5];
  pit_minv(ei, ej, M);
  pit_role_into<0>(ei, ej, M, o);
  pit_role_into<1>(ei, ej, M, o);
  pit_role_into<2>(ei, ej, M, o);
  pit_role_into<3>(ei, ej, M, o);
}

// only the mean and covariance of ei (x) ej (an entry state: ei = a prefix from block 0)
__device__ __forceinline__ void pit_combine_state(const PitEl& ei, const PitEl& ej, double (&st)[5],
                                                  double (&P)[5][5]) {
  double M[5][5], t[25], c[25];
  pit_minv(ei, ej, M);
  pit_role<1>(ei, ej, M, t);
  pit_role<2>(ei, ej, M, c);
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    st[i] = t[i];
#pragma unroll
    for (int j = i; j < 5; ++j) P[i][j] = c[pit_sy(i, j)];
  }
}

// The first pass's trajectory. A pass linearizes every sample at xbar, and where xbar is far
// from the filter's path (the start-up transient from x0, P0 = I) the fixed point is only
// reached one block per pass (scripts/study/ekf_pit_proto.py: 9 passes of crawling before
// quadratic convergence for init_m = 6 on an m = 4.3 record). So the sequential EKF runs the
// first T0 samples, their predicted states seed xbar there, and every later sample starts at
// the state entering sample T0.
__global__ __launch_bounds__(64) void ekf_pit_head_kernel(const double* __restrict__ x, int64_t nrec, int64_t rs,
                                                          int64_t T0, const double* __restrict__ x0,
                                                          const double* __restrict__ p0,
                                                          const double* __restrict__ qd,
                                                          const double* __restrict__ rv,
                                                          const double* __restrict__ wt,
                                                          double* __restrict__ hs, double* __restrict__ hst,
                                                          DfmiTrigK tk) {
  // the row form of ekf_rot_kernel (16 lanes per channel, 4 channels per wave; sin / cos by
  // rotation between anchors every 8 samples, ~2x the lane form's rate); these states only
  // seed the trajectory (the passes re-derive every sample), so a group whose arguments move
  // too far for the rotation is not rolled back here
  const int lane = threadIdx.x & 63;
  const int64_t r0 = (int64_t)blockIdx.x * 4 + (lane >> 4);
  const bool live = r0 < nrec;
  const int64_t r = live ? r0 : nrec - 1;
  int j = lane & 15;
  if (j > 4) j = 4;
  double st[5], Pc[5], qv[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    st[i] = x0[r * 5 + i];
    Pc[i] = (i == j) ? p0[i] : 0.0;
    qv[i] = (i == j) ? qd[i] : 0.0;
  }
  const double Rv = rv[r];
  const bool writer = live && (lane & 15) == 0;
  const bool odd = lane & 1;
  const RowSplitCoef rc = row_split_coef(tk, odd);
  const RotCoef ro = rot_coef(tk, odd);
  RotRegs rr;
#pragma unroll
  for (int i = 0; i < 5; ++i) rr.HP[i] = 0.0;
  rr.sth = rr.cth = rr.sa = rr.ca = rr.thp = rr.argp = rr.sd = rr.cd = 0.0;
  double dmax = 0.0;
  const double* __restrict__ xr = x + r * rs;
  // the samples 8 at a time (data and ekf_phase_kernel's w_m t_k), the next group's loads in
  // flight; the predicted state entering each sample goes to hs[r][k][5] (contiguous per
  // sample; ekf_pit_gather_kernel moves it into the block layout)
  double xc[8], wc[8];
  const int64_t T8 = T0 & ~(int64_t)7;
  if (T8 > 0) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xc[u] = xr[u];
      wc[u] = wt[u];
    }
  }
  double* __restrict__ hr = hs + r * T0 * 5;
  auto step = [&](auto rot, int64_t k, double xk, double w) {
    if (writer) {
#pragma unroll
      for (int c = 0; c < 5; ++c) hr[k * 5 + c] = st[c];
    }
    ekf_rot_step<decltype(rot)::value>(st, Pc, qv, Rv, xk, w, tk, rr, rc, ro, odd, dmax);
  };
  int64_t k = 0;
  for (; k < T8; k += 8) {
    double xn[8], wn[8];
    const int64_t kn = k + 8 < T8 ? k + 8 : k;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xn[u] = xr[kn + u];
      wn[u] = wt[kn + u];
    }
    step(std::false_type{}, k, xc[0], wc[0]);  // the anchor
#pragma unroll
    for (int u = 1; u < 8; ++u) step(std::true_type{}, k + u, xc[u], wc[u]);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xc[u] = xn[u];
      wc[u] = wn[u];
    }
  }
  for (; k < T0; ++k) step(std::false_type{}, k, xr[k], wt[k]);
  if (writer) {
#pragma unroll
    for (int c = 0; c < 5; ++c) hst[r * 5 + c] = st[c];
  }
}

// Transposes the channel data into blocks, tabulates w_m t_k (ekf_phase_kernel's
// expression: same bits), sets xbar from the head (its per-sample states below T0, the state
// entering T0 from there on) and clears the per-channel flags. One thread per (sample slot, channel); grid.y = channel.
__global__ __launch_bounds__(256) void ekf_pit_gather_kernel(const double* __restrict__ x, int64_t rs, int64_t n,
                                                             const double* __restrict__ hs,
                                                             const double* __restrict__ hst, int64_t T0, int64_t B,
                                                             int64_t nb, double w_m, double f_samp,
                                                             double* __restrict__ xt, double* __restrict__ wtt,
                                                             double* __restrict__ xbar, PitChan* __restrict__ ch,
                                                             double* __restrict__ conv, unsigned* __restrict__ done) {
  const int64_t r = blockIdx.y;
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // s = i nb + b
  const int64_t slots = B * nb;
  if (s == 0) {
    PitChan c;
    c.status = c.passes = c.stall = c.pad = 0;
    c.dprev = __builtin_nan("");
    c.rho = -1.0;
#pragma unroll
    for (int i = 0; i < kPitTrend; ++i) c.dold[i] = __builtin_nan("");
    ch[r] = c;
    conv[r] = 0.0;  // largest move of the pass (ekf_pit_blocks_kernel)
    done[r] = 0;    // workgroups of the pass kernel finished (ekf_pit_pass_kernel)
  }
  if (s >= slots) return;
  const int64_t i = s / nb, b = s - i * nb;
  const int64_t k = b * B + i;
  xt[r * slots + s] = k < n ? x[r * rs + k] : 0.0;
  if (r == 0) wtt[s] = w_m * ((double)k / f_samp);
  if (xbar) {  // the unfused path's trajectory buffer (the fused first pass reads the head itself)
    const double* src = k < T0 ? hs + (r * T0 + k) * 5 : hst + r * 5;
#pragma unroll
    for (int c = 0; c < 5; ++c) xbar[(r * 5 + c) * slots + s] = src[c];
  }
}

// The fused path's gather (no xbar): the channel data into blocks through an LDS tile of 64
// blocks x 32 samples — each block's 32 samples read as one contiguous run, each sample slot's
// 64 blocks written as one — where ekf_pit_gather_kernel reads with a stride of B samples
// (1.8 TB/s at 1,024 x 400,000 samples, B = 2,481: 3.7 ms). Also w_m t_k (z = 0) and the
// per-channel control blocks (the tile at x = y = 0). Grid (ceil(B / 32), ceil(nb / 64), nrec).
__global__ __launch_bounds__(256) void ekf_pit_gather_tiled_kernel(const double* __restrict__ x, int64_t rs,
                                                                   int64_t n, int64_t B, int64_t nb, double w_m,
                                                                   double f_samp, double* __restrict__ xt,
                                                                   double* __restrict__ wtt, PitChan* __restrict__ ch,
                                                                   double* __restrict__ conv,
                                                                   unsigned* __restrict__ done) {
  __shared__ double tile[64][33];
  const int64_t r = blockIdx.z;
  const int64_t i0 = (int64_t)blockIdx.x * 32, b0 = (int64_t)blockIdx.y * 64;
  const int t = threadIdx.x;
  if (blockIdx.x == 0 && blockIdx.y == 0 && t == 0) {
    PitChan c;
    c.status = c.passes = c.stall = c.pad = 0;
    c.dprev = __builtin_nan("");
    c.rho = -1.0;
#pragma unroll
    for (int i = 0; i < kPitTrend; ++i) c.dold[i] = __builtin_nan("");
    ch[r] = c;
    conv[r] = 0.0;
    done[r] = 0;
  }
  {  // read: thread t -> block b0 + t / 4, samples i0 + 8 (t % 4) .. + 7
    const int bl = t >> 2, il = (t & 3) * 8;
    const int64_t b = b0 + bl;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t i = i0 + il + u;
      const int64_t k = b * B + i;
      tile[bl][il + u] = (b < nb && i < B && k < n) ? x[r * rs + k] : 0.0;
    }
  }
  __syncthreads();
  const int64_t slots = B * nb;
#pragma unroll
  for (int u = 0; u < 8; ++u) {  // write: 8 sample slots x 64 blocks per pass of 256 threads
    const int e = t + 256 * u;
    const int il = e >> 6, bl = e & 63;
    const int64_t i = i0 + il, b = b0 + bl;
    if (i < B && b < nb) {
      const int64_t s = i * nb + b;
      xt[r * slots + s] = tile[bl][il];
      if (r == 0) wtt[s] = w_m * ((double)(b * B + i) / f_samp);
    }
  }
}

// Fold one sample's element (h, eps = e - h.b) into the running aggregate (see
// ekf_pit_aggregate_kernel).
__device__ __forceinline__ void pit_fold(double (&A)[25], double (&bv)[5], double (&C)[15], double (&et)[5],
                                         double (&J)[15], const double (&q)[5], double Rv, const double (&h)[5],
                                         double eps) {
  double g[5], rr[5];
#pragma unroll
  for (int i2 = 0; i2 < 5; ++i2) {
    double s2 = q[i2] * h[i2];
#pragma unroll
    for (int j = 0; j < 5; ++j) s2 = fma(C[pit_sy(i2, j)], h[j], s2);
    g[i2] = s2;
  }
  double gam = Rv;
#pragma unroll
  for (int c = 0; c < 5; ++c) gam = fma(h[c], g[c], gam);
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    double s2 = 0.0;
#pragma unroll
    for (int k = 0; k < 5; ++k) s2 = fma(A[k * 5 + c], h[k], s2);
    rr[c] = s2;
  }
  const double ig = 1.0 / gam;
  const double ei = eps * ig;
  double v[5], ri[5];
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    v[c] = g[c] * ig;
    ri[c] = rr[c] * ig;
  }
#pragma unroll
  for (int r2 = 0; r2 < 5; ++r2)
#pragma unroll
    for (int c = 0; c < 5; ++c) A[r2 * 5 + c] = fma(-v[r2], rr[c], A[r2 * 5 + c]);
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    bv[c] = fma(v[c], eps, bv[c]);
    et[c] = fma(rr[c], ei, et[c]);
  }
#pragma unroll
  for (int i2 = 0; i2 < 5; ++i2)
#pragma unroll
    for (int j = i2; j < 5; ++j) {
      const int y = pit_sy(i2, j);
      C[y] = fma(-g[i2], v[j], i2 == j ? C[y] + q[i2] : C[y]);
      J[y] = fma(ri[i2], rr[j], J[y]);
    }
}

// one sample's inputs: xbar (5), w_m t_k, y_k
struct PitSamp {
  double xb[5];
  double w, y;
};
constexpr int kPitG = 4;  // samples per prefetch group
// sample i of block b (clamped into the block: the padded slots are allocated)
// xbar == nullptr: the seeded trajectory straight from the head (ekf_pit_gather_kernel's values:
// the head's predicted state for k < T0, the state entering T0 beyond), no [r][5][slots] buffer
// (16 GB written and read at 1,024 x 400,000 samples).
__device__ __forceinline__ void pit_load_agg(PitSamp& d, const double* __restrict__ xt, const double* __restrict__ wtt,
                                             const double* __restrict__ xbar, int64_t r, int64_t slots, int64_t nb,
                                             int64_t B, int64_t b, int64_t i, const double* __restrict__ hs,
                                             const double* __restrict__ hst, int64_t T0) {
  const int64_t ii = i < B ? i : B - 1;
  const int64_t s = ii * nb + b;
  if (xbar) {
#pragma unroll
    for (int c = 0; c < 5; ++c) d.xb[c] = xbar[(r * 5 + c) * slots + s];
  } else {
    const int64_t k = b * B + ii;
    const double* src = k < T0 ? hs + (r * T0 + k) * 5 : hst + r * 5;
#pragma unroll
    for (int c = 0; c < 5; ++c) d.xb[c] = src[c];
  }
  d.w = wtt[s];
  d.y = xt[r * slots + s];
}

// Step 1 + the in-block fold of step 2: lane = block. The element of sample k (F = I,
// Q diagonal) is A_k = I - K h^T, b_k = K e, C_k = Q - (Qh)(Qh)^T / S, eta_k = h e / S,
// J_k = h h^T / S (S = h^T Q h + R, K = Q h / S, e = y_k - d_k); folding it into the
// running aggregate (A, b, C, eta, J) is the general combine with a rank-1 J_j, which
// reduces to (g = (C + Q) h, gamma = h.g + R, v = g / gamma, r = A^T h, eps = e - h.b):
//   A -= v r^T, b += v eps, C += Q - g v^T, eta += r eps / gamma, J += r r^T / gamma
// (tests/test_ekf_pit_host.py checks it against the general combine). Block 0 starts from
// the prior element (A = 0, b = x0, C = P0), the others from the identity.
__global__ __launch_bounds__(64) void ekf_pit_aggregate_kernel(const double* __restrict__ xt,
                                                               const double* __restrict__ wtt,
                                                               const double* __restrict__ xbar, int64_t n, int64_t B,
                                                               int64_t nb, const double* __restrict__ x0,
                                                               const double* __restrict__ p0,
                                                               const double* __restrict__ qd,
                                                               const double* __restrict__ rv,
                                                               const PitChan* __restrict__ ch,
                                                               double* __restrict__ agg, DfmiTrigK tk,
                                                               const double* __restrict__ hs,
                                                               const double* __restrict__ hst, int64_t T0) {
  const int64_t r = blockIdx.y;
  if (ch[r].status) return;
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const int64_t slots = B * nb;
  double A[25], bv[5], C[15], et[5], J[15], q[5];
  const bool first = b == 0;
#pragma unroll
  for (int c = 0; c < 25; ++c) A[c] = (!first && c / 5 == c % 5) ? 1.0 : 0.0;
#pragma unroll
  for (int c = 0; c < 15; ++c) C[c] = J[c] = 0.0;
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    bv[c] = first ? x0[r * 5 + c] : 0.0;
    et[c] = 0.0;
    q[c] = qd[c];
    if (first) C[pit_sy(c, c)] = p0[c];
  }
  const double Rv = rv[r];
  const int64_t kend = (b + 1) * B < n ? B : n - b * B;
  // the samples kPitG at a time, the next group's loads in flight while this one folds
  // (one wave per SIMD: nothing else hides a load's latency)
  PitSamp cur[kPitG], nxt[kPitG];
#pragma unroll
  for (int u = 0; u < kPitG; ++u) pit_load_agg(cur[u], xt, wtt, xbar, r, slots, nb, B, b, u, hs, hst, T0);
  for (int64_t i0 = 0; i0 < kend; i0 += kPitG) {
#pragma unroll
    for (int u = 0; u < kPitG; ++u)
      pit_load_agg(nxt[u], xt, wtt, xbar, r, slots, nb, B, b, i0 + kPitG + u, hs, hst, T0);
#pragma unroll
    for (int u = 0; u < kPitG; ++u) {
      if (i0 + u >= kend) break;
      const double* xb = cur[u].xb;
      const double a = xb[0], m = xb[1];
      const double th = cur[u].w + xb[3];
      double sth, cth, sa, ca;
      dfmi_sincos_k(th, tk, &sth, &cth);
      const double arg = fma(m, cth, xb[2]);
      dfmi_sincos_k(arg, tk, &sa, &ca);
      const double hv = fma(a, ca, xb[4]);
      const double h[5] = {ca, (-a * cth) * sa, -a * sa, ((a * m) * sth) * sa, 1.0};
      // eps = e - h.b with e = y - hv + h.xbar
      double eps = cur[u].y - hv;
#pragma unroll
      for (int c = 0; c < 5; ++c) eps = fma(h[c], xb[c] - bv[c], eps);
      pit_fold(A, bv, C, et, J, q, Rv, h, eps);
    }
#pragma unroll
    for (int u = 0; u < kPitG; ++u) cur[u] = nxt[u];
  }
  double* o = agg + r * kPitEl * nb + b;
#pragma unroll
  for (int c = 0; c < 25; ++c) o[(kPitA + c) * nb] = A[c];
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    o[(kPitB + c) * nb] = bv[c];
    o[(kPitE + c) * nb] = et[c];
  }
#pragma unroll
  for (int c = 0; c < 15; ++c) {
    o[(kPitC + c) * nb] = C[c];
    o[(kPitJ + c) * nb] = J[c];
  }
}

// Inclusive Hillis-Steele scan of n_el elements el[r][65][ld] in workgroups of WGE elements
// (LDS [65][WGE]), in place; the workgroup totals (the last live element's prefix) go to
// tot[r][65][gridDim.x] when tot is given: the next level of the hierarchy, scanned the same
// way until one workgroup holds a level (tot = nullptr), then made true prefixes top-down by
// ekf_pit_fixup_kernel. Padding elements are the identity. Each combine is formed by FOUR waves
// side by side, one role each (pit_role: A / b, eta / C / J; every role forms M itself):
// wave w holds elements 64 (w / 4) .. + 63 in role w % 4, so a wave never diverges and a level
// costs one role's chain (~650 fp64 instructions) instead of the whole combine's (~1,500).
template <int WGE>
__global__ __launch_bounds__(4 * WGE) void ekf_pit_scan_kernel(double* __restrict__ el, int64_t n_el, int64_t ld,
                                                               double* __restrict__ tot,
                                                               const PitChan* __restrict__ ch) {
  static_assert(WGE % 64 == 0, "whole waves per role");
  const int64_t r = blockIdx.y;
  if (ch[r].status) return;
  __shared__ double s[kPitEl * WGE];
  const int t = threadIdx.x;
  const int w = t >> 6, role = w & 3, e = ((w >> 2) << 6) + (t & 63);
  const int64_t e0 = (int64_t)blockIdx.x * WGE;
  const int64_t nlive = n_el - e0;  // live elements here (the rest: identities)
  const int span = nlive < WGE ? (int)nlive : WGE;
  double* base = el + r * kPitEl * ld + e0;
  for (int i = t; i < kPitEl * WGE; i += 4 * WGE) {
    const int c = i / WGE, k = i - c * WGE;
    s[i] = k < span ? base[c * ld + k] : pit_identity(c);
  }
  __syncthreads();
  for (int off = 1; off < span; off <<= 1) {
    double o[25];
    const bool act = e >= off && e < span;
    if (act) {
      const PitEl ei{s + e - off, WGE}, ej{s + e, WGE};
      double M[5][5];
      pit_minv(ei, ej, M);
      if (role == 0) pit_role<0>(ei, ej, M, o);
      else if (role == 1) pit_role<1>(ei, ej, M, o);
      else if (role == 2) pit_role<2>(ei, ej, M, o);
      else pit_role<3>(ei, ej, M, o);
    }
    __syncthreads();
    if (act) {
      if (role == 0) {
#pragma unroll
        for (int i = 0; i < pit_role_n<0>(); ++i) s[pit_role_comp<0>(i) * WGE + e] = o[i];
      } else if (role == 1) {
#pragma unroll
        for (int i = 0; i < pit_role_n<1>(); ++i) s[pit_role_comp<1>(i) * WGE + e] = o[i];
      } else if (role == 2) {
#pragma unroll
        for (int i = 0; i < pit_role_n<2>(); ++i) s[pit_role_comp<2>(i) * WGE + e] = o[i];
      } else {
#pragma unroll
        for (int i = 0; i < pit_role_n<3>(); ++i) s[pit_role_comp<3>(i) * WGE + e] = o[i];
      }
    }
    __syncthreads();
  }
  for (int i = t; i < kPitEl * WGE; i += 4 * WGE) {
    const int c = i / WGE, k = i - c * WGE;
    if (k < span) base[c * ld + k] = s[i];
  }
  if (tot && t < kPitEl) {
    const int64_t ng = gridDim.x;
    tot[(r * kPitEl + t) * ng + blockIdx.x] = s[t * WGE + span - 1];
  }
}

// Level l of the scan hierarchy after its own scan holds prefixes within its workgroups of
// kPitWg; element g of a later workgroup becomes the true prefix from element 0 by the
// (already true) prefix of the previous workgroups one level up: el[g] = up[g / kPitWg - 1]
// (x) el[g]. A prefix from block 0 is (0, b, C, 0, 0) (block 0's A is 0), so only b and C
// are formed (pit_combine_state). One lane per element; the hierarchy is fixed top-down.
__global__ __launch_bounds__(64) void ekf_pit_fixup_kernel(double* __restrict__ el, int64_t n_el,
                                                           const double* __restrict__ up, int64_t n_up,
                                                           const PitChan* __restrict__ ch) {
  const int64_t r = blockIdx.y;
  if (ch[r].status) return;
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + kPitWg;  // the first workgroup is exact
  if (g >= n_el) return;
  double st[5], P[5][5];
  double* e = el + r * kPitEl * n_el + g;
  pit_combine_state(PitEl{up + r * kPitEl * n_up + (g / kPitWg - 1), n_up}, PitEl{e, n_el}, st, P);
#pragma unroll
  for (int c = 0; c < 25; ++c) e[(kPitA + c) * n_el] = 0.0;
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    e[(kPitB + c) * n_el] = st[c];
    e[(kPitE + c) * n_el] = 0.0;
  }
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = i; j < 5; ++j) {
      e[(kPitC + pit_sy(i, j)) * n_el] = P[i][j];
      e[(kPitJ + pit_sy(i, j)) * n_el] = 0.0;
    }
}

// ekf_pit_fixup_kernel for the level below an UNSCANNED top of at most a few elements
// (ekf_pit_topfix): block k's elements take the prefix up[0] (x) .. (x) up[k], which lane 0
// folds left to right into LDS (k <= 3 combines) — the top level's scan launch saved.
__global__ __launch_bounds__(64) void ekf_pit_fixup_top_kernel(double* __restrict__ el, int64_t n_el,
                                                               const double* __restrict__ up, int64_t n_up,
                                                               const PitChan* __restrict__ ch) {
  const int64_t r = blockIdx.y;
  if (ch[r].status) return;
  __shared__ double pref[kPitEl];
  const int64_t k = blockIdx.x;
  const double* u = up + r * kPitEl * n_up;
  if (threadIdx.x == 0) {
    for (int c = 0; c < kPitEl; ++c) pref[c] = u[c * n_up];
    for (int64_t i = 1; i <= k; ++i) {
      double o[kPitEl];
      pit_combine(PitEl{pref, 1}, PitEl{u + i, n_up}, o);
#pragma unroll
      for (int c = 0; c < kPitEl; ++c) pref[c] = o[c];
    }
  }
  __syncthreads();
  const int64_t g = (k + 1) * kPitWg + threadIdx.x;
  if (g >= n_el) return;
  double st[5], P[5][5];
  double* e = el + r * kPitEl * n_el + g;
  pit_combine_state(PitEl{pref, 1}, PitEl{e, n_el}, st, P);
#pragma unroll
  for (int c = 0; c < 25; ++c) e[(kPitA + c) * n_el] = 0.0;
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    e[(kPitB + c) * n_el] = st[c];
    e[(kPitE + c) * n_el] = 0.0;
  }
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = i; j < 5; ++j) {
      e[(kPitC + pit_sy(i, j)) * n_el] = P[i][j];
      e[(kPitJ + pit_sy(i, j)) * n_el] = 0.0;
    }
}

// The state (x, P) entering block b: (x0, P0) for block 0, else the filtered (mean, cov)
// after block b-1 = the inclusive prefix: agg[b-1] (scanned within its workgroup) preceded by
// tot[g-1] (the scanned workgroup totals) when b-1 lies past the first workgroup.
__device__ __forceinline__ void pit_entry(int64_t r, int64_t b, int64_t nb, const double* __restrict__ x0,
                                          const double* __restrict__ p0, const double* __restrict__ agg,
                                          const double* __restrict__ tot, double (&st)[5], double (&P)[5][5]) {
  if (b == 0) {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      st[i] = x0[r * 5 + i];
#pragma unroll
      for (int j = 0; j < 5; ++j) P[i][j] = (i == j) ? p0[i] : 0.0;
    }
  } else {
    const int64_t p = b - 1, g = p / kPitWg;
    const PitEl loc{agg + r * kPitEl * nb + p, nb};
    if (g == 0) {
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        st[i] = loc(kPitB + i);
#pragma unroll
        for (int j = i; j < 5; ++j) P[i][j] = loc.C(i, j);
      }
    } else {
      const int64_t ng = (nb + kPitWg - 1) / kPitWg;
      pit_combine_state(PitEl{tot + r * kPitEl * ng + (g - 1), ng}, loc, st, P);
    }
  }
}

// Step 3: lane = block. Entry state: (x0, P0) for block 0; else the filtered (mean, cov)
// after block b-1, i.e. the inclusive prefix: agg[b-1] (scanned within its workgroup)
// preceded by tot[g-1] (scanned workgroup totals) when b-1 lies past the first workgroup.
// Then ekf_step over the block (the lane kernel's arithmetic), writing the next xbar (the
// state entering each following sample), its largest relative move into conv[r] (max over
// the channel's blocks) and the snapshots (fitters.py:305-307).
__global__ __launch_bounds__(64) void ekf_pit_blocks_kernel(const double* __restrict__ xt,
                                                            const double* __restrict__ wtt,
                                                            double* __restrict__ xbar, int64_t n, int64_t B, int64_t nb,
                                                            const double* __restrict__ x0,
                                                            const double* __restrict__ p0,
                                                            const double* __restrict__ qd,
                                                            const double* __restrict__ rv,
                                                            const double* __restrict__ agg,
                                                            const double* __restrict__ tot, const PitChan* __restrict__ ch,
                                                            double* __restrict__ conv, int R, int64_t nbuf,
                                                            double* __restrict__ states, int measure, DfmiTrigK tk) {
  const int64_t r = blockIdx.y;
  if (ch[r].status) return;
  const int64_t b0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = b0 < nb;  // lanes past the last block stay for the wave's max (no work)
  const int64_t b = live ? b0 : nb - 1;
  const int64_t slots = B * nb;
  double st[5], P[5][5], Q[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) Q[i] = qd[i];
  pit_entry(r, b, nb, x0, p0, agg, tot, st, P);
  const double Rv = rv[r];
  double dmax = 0.0, dsnap = 0.0;
  const int64_t kend = !live ? 0 : (b + 1) * B < n ? B : n - b * B;
  // inputs kPitG samples ahead (see ekf_pit_aggregate_kernel): y_k, w_m t_k and the xbar of
  // sample k + 1 this block overwrites
  PitSamp cur[kPitG], nxt[kPitG];
  auto load = [&](PitSamp& d, int64_t i) {
    const int64_t ic = i < B ? i : B - 1;
    const int64_t s = ic * nb + b, s1 = ic + 1 < B ? s + nb : b + 1;  // slot of sample k + 1
    d.w = wtt[s];
    d.y = xt[r * slots + s];
#pragma unroll
    for (int c = 0; c < 5; ++c) d.xb[c] = xbar[(r * 5 + c) * slots + s1];
  };
#pragma unroll
  for (int u = 0; u < kPitG; ++u) load(cur[u], u);
  for (int64_t i0 = 0; i0 < kend; i0 += kPitG) {
#pragma unroll
    for (int u = 0; u < kPitG; ++u) load(nxt[u], i0 + kPitG + u);
#pragma unroll
    for (int u = 0; u < kPitG; ++u) {
      const int64_t i = i0 + u;
      if (i >= kend) break;
      ekf_step(st, P, Q, Rv, cur[u].y, cur[u].w, tk);
      const int64_t k = b * B + i;
      if (k + 1 < n) {
        const int64_t s1 = i + 1 < B ? i * nb + b + nb : b + 1;
#pragma unroll
        for (int c = 0; c < 5; ++c) {
          const double d = fabs(st[c] - cur[u].xb[c]) / fmax(1.0, fabs(st[c]));
          dmax = d <= dmax ? dmax : d;  // NaN propagates (never "converged")
          xbar[(r * 5 + c) * slots + s1] = st[c];
        }
      }
      if ((k + 1) % R == 0) {
        const int64_t bi = (k + 1) / R - 1;
        if (bi < nbuf) pit_snapshot(states + (r * nbuf + bi) * 5, st, dsnap);
      }
    }
#pragma unroll
    for (int u = 0; u < kPitG; ++u) cur[u] = nxt[u];
  }
  if (measure == 0) dmax = dsnap;
  // the channel's largest move: a non-negative double (or NaN, above every finite value
  // and inf) orders as its bits, so the wave's max goes to conv[r] by one integer atomic
  unsigned long long bits = __builtin_bit_cast(unsigned long long, dmax);
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const unsigned long long o = __shfl_xor(bits, w, 64);
    bits = o > bits ? o : bits;
  }
  if ((threadIdx.x & 63) == 0) atomicMax((unsigned long long*)conv + r, bits);
}

// Steps 3 and 1 of the next pass in one kernel (the default): lane = block runs the true EKF
// from its entry state (pit_entry over the scan in agg / tot) and folds every sample's element
// into the block's next aggregate (agg_out, scanned next) as it goes. The element of sample k
// is linearized at the state entering k — the EKF step's own predicted state, whose H and
// h(x) ekf_step_h has just formed — so the fold costs only the rank-1 update, and no
// trajectory is written or re-read. Convergence: the entry state's largest relative move
// since the previous pass (ent, NaN before the first) into conv[r] as in
// ekf_pit_blocks_kernel. Snapshots as there.
__global__ __launch_bounds__(64) void ekf_pit_pass_kernel(const double* __restrict__ xt,
                                                          const double* __restrict__ wtt, int64_t n, int64_t B,
                                                          int64_t nb, const double* __restrict__ x0,
                                                          const double* __restrict__ p0,
                                                          const double* __restrict__ qd,
                                                          const double* __restrict__ rv,
                                                          const double* __restrict__ agg,
                                                          const double* __restrict__ tot,
                                                          double* __restrict__ agg_out, double* __restrict__ ent,
                                                          PitChan* __restrict__ ch, double* __restrict__ conv,
                                                          unsigned* __restrict__ done, PitRule rule, double* __restrict__ hist, int R,
                                                          int64_t nbuf, double* __restrict__ states,
                                                          DfmiTrigK tk) {
  const int64_t r = blockIdx.y;
  if (ch[r].status) return;
  const int64_t b0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = b0 < nb;  // lanes past the last block stay for the wave's max (no work)
  const int64_t b = live ? b0 : nb - 1;
  const int64_t slots = B * nb;
  double st[5], P[5][5], Q[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) Q[i] = qd[i];
  pit_entry(r, b, nb, x0, p0, agg, tot, st, P);
  double dmax = 0.0;
  if (live && rule.measure == 1) {
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      double* pe = ent + (r * 5 + c) * nb + b;
      const double d = fabs(st[c] - *pe) / fmax(1.0, fabs(st[c]));
      dmax = d <= dmax ? dmax : d;  // NaN (the first pass) propagates: never "converged"
      *pe = st[c];
    }
  }
  // the block's next aggregate: block 0 from the prior element, the others from the identity
  double A[25], bv[5], C[15], et[5], J[15];
  double dsnap = 0.0;
  const bool first = b == 0;
#pragma unroll
  for (int c = 0; c < 25; ++c) A[c] = (!first && c / 5 == c % 5) ? 1.0 : 0.0;
#pragma unroll
  for (int c = 0; c < 15; ++c) C[c] = J[c] = 0.0;
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    bv[c] = first ? x0[r * 5 + c] : 0.0;
    et[c] = 0.0;
    if (first) C[pit_sy(c, c)] = p0[c];
  }
  const double Rv = rv[r];
  const int64_t kend = !live ? 0 : (b + 1) * B < n ? B : n - b * B;
  double yc[kPitG], wc[kPitG], yn[kPitG], wn[kPitG];
  auto load = [&](double& y, double& w, int64_t i) {
    const int64_t s = (i < B ? i : B - 1) * nb + b;
    w = wtt[s];
    y = xt[r * slots + s];
  };
#pragma unroll
  for (int u = 0; u < kPitG; ++u) load(yc[u], wc[u], u);
  for (int64_t i0 = 0; i0 < kend; i0 += kPitG) {
#pragma unroll
    for (int u = 0; u < kPitG; ++u) load(yn[u], wn[u], i0 + kPitG + u);
#pragma unroll
    for (int u = 0; u < kPitG; ++u) {
      const int64_t i = i0 + u;
      if (i >= kend) break;
      double xp[5], H[5], hv;
#pragma unroll
      for (int c = 0; c < 5; ++c) xp[c] = st[c];
      ekf_step_h(st, P, Q, Rv, yc[u], wc[u], tk, H, hv);
      // eps = e - h.b with e = y - hv + h.xbar, xbar = the predicted state
      double eps = yc[u] - hv;
#pragma unroll
      for (int c = 0; c < 5; ++c) eps = fma(H[c], xp[c] - bv[c], eps);
      pit_fold(A, bv, C, et, J, Q, Rv, H, eps);
      const int64_t k = b * B + i;
      if ((k + 1) % R == 0) {
        const int64_t bi = (k + 1) / R - 1;
        if (bi < nbuf) pit_snapshot(states + (r * nbuf + bi) * 5, st, dsnap);
      }
    }
#pragma unroll
    for (int u = 0; u < kPitG; ++u) {
      yc[u] = yn[u];
      wc[u] = wn[u];
    }
  }
  if (live) {
    double* o = agg_out + r * kPitEl * nb + b;
#pragma unroll
    for (int c = 0; c < 25; ++c) o[(kPitA + c) * nb] = A[c];
#pragma unroll
    for (int c = 0; c < 5; ++c) {
      o[(kPitB + c) * nb] = bv[c];
      o[(kPitE + c) * nb] = et[c];
    }
#pragma unroll
    for (int c = 0; c < 15; ++c) {
      o[(kPitC + c) * nb] = C[c];
      o[(kPitJ + c) * nb] = J[c];
    }
  }
  if (rule.measure == 0) dmax = dsnap;
  unsigned long long bits = __builtin_bit_cast(unsigned long long, dmax);
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const unsigned long long o = __shfl_xor(bits, w, 64);
    bits = o > bits ? o : bits;
  }
  // the channel's check (ekf_pit_check_kernel's, without a launch): the last workgroup of
  // the channel to finish (one wave each: lane 0 made the atomicMax) reads the max and applies
  // the stop rule; every other workgroup of this launch had passed its status test by then
  if (threadIdx.x == 0) {
    atomicMax((unsigned long long*)conv + r, bits);
    __threadfence();
    if (atomicAdd(done + r, 1u) == gridDim.x - 1) {
      __threadfence();
      const double c = __builtin_bit_cast(double, atomicAdd((unsigned long long*)conv + r, 0ull));
      pit_decide(ch[r], c, rule, hist ? hist + r * rule.hist_n : nullptr);
      atomicExch((unsigned long long*)conv + r, 0ull);
      atomicExch(done + r, 0u);
    }
  }
}

// One thread per channel (the unfused path): the stop rule on the pass's largest move of xbar
// (ekf_pit_blocks_kernel), then conv cleared for the next pass.
__global__ __launch_bounds__(64) void ekf_pit_check_kernel(double* __restrict__ conv, int64_t nrec, PitRule rule,
                                                           PitChan* __restrict__ ch, double* __restrict__ hist) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrec || ch[r].status) return;
  pit_decide(ch[r], conv[r], rule, hist ? hist + r * rule.hist_n : nullptr);
  conv[r] = 0.0;
}

// Channels the passes handed to the sequential kernel since the previous call: status 2 (with
// final != 0: every channel not converged, status 0 at the pass cap included) and not yet flagged
// in `handed`, appended to idx[0..] in channel order (ballot prefix: one wave, no atomics). The
// sequential kernels then read those records in place through idx (no copy of the samples), on
// a stream of their own while the other channels keep passing (dfmi_capi.hip ekf_pit_run).
__global__ __launch_bounds__(64) void ekf_pit_handover_kernel(const PitChan* __restrict__ ch, int64_t nrec,
                                                              unsigned* __restrict__ handed, int* __restrict__ idx,
                                                              int final_) {
  const int lane = threadIdx.x;
  int base = 0;
  for (int64_t r0 = 0; r0 < nrec; r0 += 64) {
    const int64_t r = r0 + lane;
    bool take = false;
    if (r < nrec) {
      const int s = ch[r].status;
      take = handed[r] == 0u && (s == 2 || (final_ && s != 1));
    }
    const uint64_t m = __ballot(take);
    if (take) {
      idx[base + __popcll(m & ((1ull << lane) - 1ull))] = (int)r;
      handed[r] = 1u;
    }
    base += __popcll(m);
  }
}

}  // namespace dfmi
