// lm.h — per-segment Levenberg–Marquardt kernel for gfx950 (fp64).
//
// Reference (file:line in /root/reference):
//   coeffs ................... fit.py:68-150   -> eval_reg / eval_gen (FULL)
//   ssqf ..................... fit.py:152-167  -> the ssq of the same evaluation
//   msolve ................... fit.py:169-206  -> damped_solve
//   _run_lma_fit ............. fit.py:208-258  -> lm_descend
//   _find_best_initial_guess . fit.py:260-320  -> m_grid_seed
//   fit ...................... fit.py:322-361  -> fit_segment
//   _process_fit_chunk ....... fitters.py:13-60 (warm start inside a chunk) -> lm_chunks_kernel
//
// Mapping: ONE LANE OWNS ONE CHUNK (a run of segments fitted with a warm-start
// chain, np.array_split semantics). With chunk size 1 — the default GPU mode —
// every lane fits one segment, so a wave fits 64 segments at once with no
// cross-lane traffic; the 4-parameter problem (2·ndata residuals, J^T J, J^T r,
// the damped 4×4 solve) lives in that lane's registers. QI is stored
// component-major (qi[c·ld + s]) so a wave loads each component coalesced.
//
// Two code paths, chosen per launch from ndata:
//  * register path (ndata <= NDMAX, NDMAX = 12 or 16): the model's structure is
//    used to cut the work per evaluation (see "Register path" below): J_0..J_{NDMAX+1}(m)
//    from ONE backward Miller pass, cos/sin(j psi) by rotation (psi_rotate), the
//    J^T J / J^T r sums in closed per-harmonic form (the psi column is orthogonal
//    to the other three: J^T J is block-diagonal, so the damped solve is a 3x3 LDL^T
//    plus one division), branch-free Cody-Waite sincos.
//  * general path (any ndata, e.g. 30/62): the two-pass Miller walk of
//    dfmi_math.h hands out J values in descending order, nothing is stored; the
//    literal per-residual Jacobian and the pivoting 4x4 solve (msolve's dgesv).
// The reference recomputes coeffs() at an accepted trial point (fit.py:250-251);
// here that is the trial's stored Bessel values and trig plus the Jacobian part.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "dfmi_math.h"

namespace dfmi {

constexpr int kMaxLambda = 16;

struct LMConst {
  int max_steps;             // fit.py:7
  int n_lambda;              // fit.py:222
  double lambdas[kMaxLambda];
  double min_step_norm;      // fit.py:230 (1e-15)
  double conv_improve;       // fit.py:8
  double conv_param_change;  // fit.py:9
  double fitok_threshold;    // fit.py:10
  double bessel_amp_thr;     // fit.py:15
  double sincos_amp_thr;     // fit.py:16
  int n_grid;                // len(np.arange(M_GRID_MIN, M_GRID_MAX + M_GRID_STEP, M_GRID_STEP))
  double grid_min;           // fit.py:12
  double grid_delta;         // (min + step) - min, numpy arange fill
  DfmiTrigK trig;            // dfmi_sincos_k's constants (in SGPRs as part of the kernel argument)
};

#define DFMI_HDI __host__ __device__ __forceinline__

// cos(phi + j*pi/2) from (cos phi, sin phi): j mod 4 -> c, -s, -c, s
DFMI_HDI double quarter_turn(int j, double c, double s) {
  switch (j & 3) {
    case 0: return c;
    case 1: return -s;
    case 2: return -c;
    default: return s;
  }
}

struct Eval {
  double ssq;
  double a00, a01, a02, a03, a11, a12, a13, a22, a23, a33;  // J^T J (upper)
  double g0, g1, g2, g3;                                   // J^T r
};

// One harmonic's contribution (fit.py:110-148 for harmonic j).
DFMI_HDI void harmonic_term(Eval& e, int j, double a, bool a_nz, double cph, double sph, double Jm1, double J0,
                            double Jp1, double cj, double sj, double Q, double I) {
  const double pt = quarter_turn(j, cph, sph);       // cos(phi + j pi/2)
  const double ptd = quarter_turn(j + 1, cph, sph);  // cos(phi + j pi/2 + pi/2)
  const double common = a * pt * J0;
  const double rq = fma(-common, cj, Q);  // Q - model_Q (model_Q = common cos(j psi))
  const double ri = fma(common, sj, I);   // I - model_I (model_I = -common sin(j psi))
  e.ssq = fma(rq, rq, e.ssq);
  e.ssq = fma(ri, ri, e.ssq);
  // d model / d a = model / a (fit.py:126-128), written without the division
  const double base = pt * J0;
  const double q0 = a_nz ? base * cj : 0.0;
  const double i0 = a_nz ? -base * sj : 0.0;
  const double dJ = 0.5 * (Jm1 - Jp1);
  const double cm = a * pt * dJ;
  const double q1 = cm * cj, i1 = -cm * sj;
  const double cphi = a * ptd * J0;
  const double q2 = cphi * cj, i2 = -cphi * sj;
  const double q3 = common * -sj * (double)j, i3 = -common * cj * (double)j;
  e.a00 += q0 * q0 + i0 * i0;
  e.a01 += q0 * q1 + i0 * i1;
  e.a02 += q0 * q2 + i0 * i2;
  e.a03 += q0 * q3 + i0 * i3;
  e.a11 += q1 * q1 + i1 * i1;
  e.a12 += q1 * q2 + i1 * i2;
  e.a13 += q1 * q3 + i1 * i3;
  e.a22 += q2 * q2 + i2 * i2;
  e.a23 += q2 * q3 + i2 * i3;
  e.a33 += q3 * q3 + i3 * i3;
  e.g0 += q0 * rq + i0 * ri;
  e.g1 += q1 * rq + i1 * ri;
  e.g2 += q2 * rq + i2 * ri;
  e.g3 += q3 * rq + i3 * ri;
}

DFMI_HDI void eval_zero(Eval& e) { e = Eval{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; }

// ---------------------------------------------------------------------------
// Register path
// ---------------------------------------------------------------------------

// 1/d to within an ulp or two: v_rcp_f64 + two Newton steps on the device (the
// IEEE division sequence costs ~3x the instructions); exact division on the host. Two
// Newton steps are not guaranteed to round correctly, so the device and the host build
// of this header (tests/hostcheck) may differ by an ulp in 2/x, 1/S and hence in J_k:
// an ulp-level deviation from the host / oracle builds by design, counted by
// tests/test_gpu_numerics.py::test_device_bessel_regs_vs_host_build (how many J_k differ,
// max ulps); the fits' parity with the reference is gated by the record tests.
DFMI_HDI double rcp_nr(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  r = fma(r, fma(-d, r, 1.0), r);
  return r;
#else
  return 1.0 / d;
#endif
}

// J_0..J_{NB-1}(x) into registers with one backward Miller pass.
// |x| < 1e-3 takes the power series (4 terms, relative error < 1e-20); above
// that the unrolled low-order part of the pass (orders < NB <= 18) grows by at
// most ~1e70, so only the runtime part of the pass (orders >= NB) carries the
// exact power-of-two rescaling of dfmi_math.h.
// dfmi_bessel_j01_large out of line on the device: inlined, its ~30 polynomial constants and
// the sincos are hoisted into registers across the LM kernels and push lm_chunks_kernel from
// 248 VGPRs (2 waves per SIMD) to 256 + 34 AGPRs (1 wave); as a call on this rare branch
// (|m| >= 64: runaway descents) the hot path keeps its allocation.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(DFMI_BES_LARGE_INLINE)
__device__ __attribute__((noinline)) void bessel_j01_large_ool(double ax, double* j0, double* j1) {
  dfmi_bessel_j01_large(ax, j0, j1);
}
DFMI_HDI void bessel_j01_large_call(double ax, double& j0, double& j1) { bessel_j01_large_ool(ax, &j0, &j1); }
#else
DFMI_HDI void bessel_j01_large_call(double ax, double& j0, double& j1) { dfmi_bessel_j01_large(ax, &j0, &j1); }
#endif

template <int NB>
DFMI_HDI void bessel_regs(double x, int N, double (&J)[NB]) {
  const double ax = fabs(x);
  if (!(ax < 1.0e5)) {  // NaN / absurd argument
#pragma unroll
    for (int k = 0; k < NB; ++k) J[k] = __builtin_nan("");
    return;
  }
  if (ax < 1.0e-3) {  // includes x == 0 (J_0 = 1, J_k = 0)
    const double h = 0.5 * x, q = h * h;
    double t = 1.0;  // (x/2)^k / k!
#pragma unroll
    for (int k = 0; k < NB; ++k) {
      if (k > 0) t *= h * (1.0 / (double)k);  // compile-time reciprocals: no fp64 division
      const double r1 = 1.0 / (double)(k + 1), r2 = 1.0 / (2.0 * (k + 2)), r3 = 1.0 / (3.0 * (k + 3));
      // 1 - q/(k+1) + q^2/(2(k+1)(k+2)) - q^3/(6(k+1)(k+2)(k+3))
      const double s = 1.0 - q * r1 * (1.0 - q * r2 * (1.0 - q * r3));
      J[k] = t * s;
    }
    return;
  }
  static_assert((NB & 1) == 0, "the pair loop below needs an even NB");
  if (dfmi_bessel_use_large(ax, NB - 1)) {  // runaway descents: O(NB), not ~1.1|x| orders (dfmi_math.h)
    double j0, j1;
    bessel_j01_large_call(ax, j0, j1);
    const double tox = 2.0 * rcp_nr(ax);
    J[0] = j0;
    J[1] = j1;
#pragma unroll
    for (int k = 1; k < NB - 1; ++k) J[k + 1] = fma((double)k * tox, J[k], -J[k - 1]);
#pragma unroll
    for (int k = 1; k < NB; k += 2) J[k] = x < 0.0 ? -J[k] : J[k];  // J_k(-x) = (-1)^k J_k(x)
    return;
  }
  int M = dfmi_bessel_start(N, ax);
  if (M < NB) M = (NB + 1) & ~1;
  const double tox = 2.0 * rcp_nr(ax);
  // Runtime part of the pass without the per-order overflow test: power-of-two
  // rescaling is exact, so a pass that never leaves the finite range gives the same
  // bits as the rescaled one; only if it overflowed does the checked pass run.
  // Orders k = M .. NB (M, NB even) in pairs (k even: f_{k-1}, no S term; k - 1 odd:
  // f_{k-2}, S += 2 f_{k-2}), k held as an exact double counter: the same operations
  // as one order per iteration with (double)k (bit for bit), without the per-order int
  // conversion, parity select and register rotation (12 -> 4.5 VALU per order).
  double fp1 = 0.0, f = 1.0, S = 2.0;  // order M (even) contributes 2 f_M
  {
    double kd = (double)M;
    for (int i = (M - NB) >> 1; i > 0; --i) {
      const double a = fma(kd * tox, f, -fp1);         // f_{k-1}
      const double b = fma((kd - 1.0) * tox, a, -f);   // f_{k-2}
      S = fma(2.0, b, S);
      fp1 = a;
      f = b;
      kd -= 2.0;
    }
    const double a = fma(kd * tox, f, -fp1);  // k = NB: f_{NB-1}
    fp1 = f;
    f = a;
  }
  if (!(fabs(f) < 1.0e300) || !(fabs(S) < 1.0e300)) {
    const double big = ldexp(1.0, DFMI_BES_BIG_EXP);
    fp1 = 0.0;
    f = 1.0;
    S = 2.0;
    for (int k = M; k >= NB; --k) {
      double fm1 = fma((double)k * tox, f, -fp1);
      if (fabs(fm1) > big) {
        fm1 = ldexp(fm1, -DFMI_BES_BIG_EXP);
        f = ldexp(f, -DFMI_BES_BIG_EXP);
        S = ldexp(S, -DFMI_BES_BIG_EXP);
      }
      if (((k - 1) & 1) == 0) S += 2.0 * fm1;
      fp1 = f;
      f = fm1;
    }
  }
  J[NB - 1] = f;
#pragma unroll
  for (int k = NB - 1; k >= 1; --k) {
    const double fm1 = fma((double)k * tox, f, -fp1);
    J[k - 1] = fm1;
    if (k - 1 == 0) S += fm1;
    else if (((k - 1) & 1) == 0) S += 2.0 * fm1;
    fp1 = f;
    f = fm1;
  }
  const double invS = rcp_nr(S);
  const double invS_odd = x < 0.0 ? -invS : invS;  // J_k(-x) = (-1)^k J_k(x): same bits as negating J_k invS
#pragma unroll
  for (int k = 0; k < NB; ++k) J[k] *= (k & 1) ? invS_odd : invS;
}

// Structure of the model (fit.py:68-150) per harmonic j, with P = cos(phi + j pi/2),
// D = cos(phi + j pi/2 + pi/2), c = a P J_j, dJ = (J_{j-1} - J_{j+1}) / 2 and
// (cj, sj) = (cos j psi, sin j psi):
//   residuals    rq = Q_j - c cj,  ri = I_j + c sj
//   Jacobian     d/d(a, m, phi) of (model_Q, model_I) = u_k (cj, -sj),
//                u = (P J_j [0 if a == 0: fit.py:126-128], a P dJ, a D J_j);
//                d/dpsi = -j c (sj, cj)
// hence, with w = cj^2 + sj^2 (= 1 up to rounding):
//   (J^T J)_kl = sum u_k u_l w (k, l < 3),  (J^T J)_33 = sum (j c)^2 w,
//   (J^T J)_k3 = 0 exactly (the psi column is orthogonal to the others),
//   (J^T r)_k  = sum u_k (cj rq - sj ri),   (J^T r)_3 = -sum j c (sj rq + cj ri).
// The reference forms J^T J by a BLAS product of the 2 ndata x 4 Jacobian, whose k3
// entries are rounding residue (~1e-17 of the diagonal); the solve below treats them
// as the zeros they are. Differences to the literal evaluation: rounding only (the
// register path agrees with the literal general path within the parity tolerances,
// tests/test_host_numerics.py).
// Scheduling fence between the unrolled harmonics of the register path: without it the
// machine scheduler hoists every harmonic's products ahead of the accumulations (the
// J^T J pass then held ~190 VGPRs, pushing the LM kernel to one wave per SIMD).
#if defined(__HIP_DEVICE_COMPILE__)
#define DFMI_HARMONIC_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define DFMI_HARMONIC_FENCE() ((void)0)
#endif

// Register-path variant tags: NDMAX = n (any ndata <= n, harmonics above ndata masked)
// or kExactNd | n (ndata == n exactly: no masking; dispatched for the default 10).
constexpr int kExactNd = 1 << 8;
constexpr int nd_cap(int v) { return v & (kExactNd - 1); }
constexpr bool nd_exact(int v) { return (v & kExactNd) != 0; }

// (cos, sin)(j psi) -> (cos, sin)((j+1) psi): rotation through (c1, s1) = (cos, sin)(psi),
// 2 mul + 2 fma. Not the two-fma Chebyshev recurrence (cos((j+1)psi) = 2 cos psi cos(j psi) -
// cos((j-1)psi)): at the fitted |psi| ~ 1e-4 its two characteristic roots e^{+-i psi} nearly
// coincide and its rounding errors grow ~ j^2; measured on 200 config-2 minima, the error of
// ssqf(p + 1e-9) - ssqf(p) against a 40-digit evaluation was 3.9e-20 rms with it, 6.3e-21 with
// the rotation, 2.1e-20 for the reference's numpy / scipy evaluation. That difference is what
// the LM's accept test (ssq_try < ssq0, fit.py:240) resolves for the last sub-1e-9 steps, so
// the recurrence's noise decided where the register path stopped.
DFMI_HDI void psi_rotate(double& cj, double& sj, double c1, double s1) {
  const double cn = fma(cj, c1, -(sj * s1));
  const double sn = fma(sj, c1, cj * s1);
  cj = cn;
  sj = sn;
}

template <int V>
struct TrialReg {
  double J[nd_cap(V) + 2];
  double cph, sph, c1, s1, ssq;
};

// QI of harmonic j (1-based) for the unrolled loops: every load is issued
// unconditionally (no per-harmonic branch: a branch around each load serialises the
// loads' latency), from a clamped index, and masked to 0 above ndata.
template <int V, typename QF>
DFMI_HDI void qi_pair(const QF& q, int nd, int j, double& Q, double& I) {
  if constexpr (nd_exact(V)) {
    Q = q.qc(j - 1);
    I = q.qs(j - 1);
  } else {
    const bool on = j <= nd;
    const int h = on ? j - 1 : 0;
    const double qv = q.qc(h), iv = q.qs(h);
    Q = on ? qv : 0.0;
    I = on ? iv : 0.0;
  }
}

// 1.0 for harmonics j <= ndata, 0.0 above (masks the model terms of the unrolled loops)
template <int V>
DFMI_HDI double hmask(int nd, int j) {
  if constexpr (nd_exact(V)) return 1.0;
  else return j <= nd ? 1.0 : 0.0;
}

// ssqf (fit.py:152-167) at p; keeps the point's Bessel values and trig in t for the
// Jacobian of an accepted trial (eval_reg_accept). Harmonics accumulate into two
// partial sums (odd / even j): two independent fma chains.
template <int V, typename QF>
DFMI_HDI double eval_reg_trial(const QF& q, int nd, const double (&p)[4], TrialReg<V>& t, const DfmiTrigK& k) {
  constexpr int NDMAX = nd_cap(V);
  double Q[NDMAX], I[NDMAX];
#pragma unroll
  for (int j = 1; j <= NDMAX; ++j) qi_pair<V>(q, nd, j, Q[j - 1], I[j - 1]);
  dfmi_sincos_auto(p[2], k, &t.sph, &t.cph);
  dfmi_sincos_auto(p[3], k, &t.s1, &t.c1);
  bessel_regs<NDMAX + 2>(p[1], nd_exact(V) ? NDMAX + 1 : nd + 1, t.J);
  const double ac = p[0] * t.cph, as = p[0] * t.sph;
  double so = 0.0, se = 0.0;
  double cj = t.c1, sj = t.s1;  // (cos, sin)(j psi)
#pragma unroll
  for (int j = 1; j <= NDMAX; ++j) {
    const double c = quarter_turn(j, ac, as) * t.J[j] * hmask<V>(nd, j);  // a cos(phi + j pi/2) J_j
    const double rq = fma(-c, cj, Q[j - 1]);
    const double ri = fma(c, sj, I[j - 1]);
    double& acc = (j & 1) ? so : se;
    acc = fma(rq, rq, acc);
    acc = fma(ri, ri, acc);
    // cos / sin((j+1) psi) by rotation through psi (see psi_rotate)
    psi_rotate(cj, sj, t.c1, t.s1);
  }
  t.ssq = so + se;
  return t.ssq;
}

// coeffs (fit.py:68-150) at the trial point of t: J^T J and J^T r in the closed form
// above; e.ssq is the trial's.
template <int V, typename QF>
DFMI_HDI void eval_reg_accept(const QF& q, int nd, const double (&p)[4], const TrialReg<V>& t, Eval& e) {
  constexpr int NDMAX = nd_cap(V);
  double Q[NDMAX], I[NDMAX];
#pragma unroll
  for (int j = 1; j <= NDMAX; ++j) qi_pair<V>(q, nd, j, Q[j - 1], I[j - 1]);
  const double a = p[0];
  const double ac = a * t.cph, as = a * t.sph;
  // d model / d a = 0 at a == 0 (fit.py:126-128): a select, not a branch (a branch here
  // splits the pass in two and keeps every harmonic's temporaries live across it)
  const double cph0 = (a != 0.0) ? t.cph : 0.0, sph0 = (a != 0.0) ? t.sph : 0.0;
  double a00 = 0.0, a01 = 0.0, a02 = 0.0, a11 = 0.0, a12 = 0.0, a22 = 0.0, a33 = 0.0;
  double g0 = 0.0, g1 = 0.0, g2 = 0.0, g3 = 0.0;
  double cj = t.c1, sj = t.s1;
#pragma unroll
  for (int j = 1; j <= NDMAX; ++j) {
    const double Jj = t.J[j] * hmask<V>(nd, j);  // 0 above ndata: every term below vanishes
    const double aP = quarter_turn(j, ac, as), aD = quarter_turn(j + 1, ac, as);
    const double c = aP * Jj;
    const double u0 = quarter_turn(j, cph0, sph0) * Jj;
    const double u1 = aP * (0.5 * (t.J[j - 1] - t.J[j + 1])) * hmask<V>(nd, j);
    const double u2 = aD * Jj;
    const double rq = fma(-c, cj, Q[j - 1]);
    const double ri = fma(c, sj, I[j - 1]);
    const double A = fma(cj, rq, -(sj * ri));
    const double B = fma(sj, rq, cj * ri);
    const double w = fma(cj, cj, sj * sj);
    const double v0 = u0 * w, v1 = u1 * w, v2 = u2 * w;
    a00 = fma(v0, u0, a00);
    a01 = fma(v0, u1, a01);
    a02 = fma(v0, u2, a02);
    a11 = fma(v1, u1, a11);
    a12 = fma(v1, u2, a12);
    a22 = fma(v2, u2, a22);
    const double jc = (double)j * c;
    a33 = fma(jc * w, jc, a33);
    g0 = fma(u0, A, g0);
    g1 = fma(u1, A, g1);
    g2 = fma(u2, A, g2);
    g3 = fma(-jc, B, g3);
    psi_rotate(cj, sj, t.c1, t.s1);
    DFMI_HARMONIC_FENCE();
  }
  e = Eval{t.ssq, a00, a01, a02, 0.0, a11, a12, 0.0, a22, 0.0, a33, g0, g1, g2, g3};
}

// msolve (fit.py:169-206) for the register path's block-diagonal J^T J: the (a, m, phi)
// block by LDL^T (symmetric positive semi-definite: no pivoting needed), psi by one
// division. numpy raises LinAlgError -> dp = 0 when dgesv meets an exactly-zero
// pivot; the block form meets an exactly-zero pivot in the same structural cases
// (a = 0 or m = 0: whole rows of J^T J vanish), tested by the edge vectors of
// tests/golden/lm_vectors.npz.
DFMI_HDI void damped_solve_block(const Eval& e, double lam, double (&dp)[4]) {
  const double d0 = fma(lam, e.a00, e.a00);
  const double A11 = fma(lam, e.a11, e.a11), A22 = fma(lam, e.a22, e.a22), A33 = fma(lam, e.a33, e.a33);
  const double r0 = rcp_nr(d0);
  const double l10 = e.a01 * r0, l20 = e.a02 * r0;
  const double d1 = fma(-l10, e.a01, A11);
  const double r1 = rcp_nr(d1);
  const double t21 = fma(-l20, e.a01, e.a12);
  const double l21 = t21 * r1;
  const double d2 = fma(-l21, t21, fma(-l20, e.a02, A22));
  const double r2 = rcp_nr(d2);
  const double y1 = fma(-l10, e.g0, e.g1);
  const double y2 = fma(-l21, y1, fma(-l20, e.g0, e.g2));
  const double x2 = y2 * r2;
  const double x1 = fma(-l21, x2, y1 * r1);
  const double x0 = fma(-l20, x2, fma(-l10, x1, e.g0 * r0));
  const double x3 = e.g3 * rcp_nr(A33);
  const bool singular = (d0 == 0.0) || (d1 == 0.0) || (d2 == 0.0) || (A33 == 0.0);
  dp[0] = singular ? 0.0 : x0;
  dp[1] = singular ? 0.0 : x1;
  dp[2] = singular ? 0.0 : x2;
  dp[3] = singular ? 0.0 : x3;
}

// ---------------------------------------------------------------------------
// General path: QI from global memory, two-pass Bessel walk (descending j).
// ---------------------------------------------------------------------------
template <typename Body>
DFMI_HDI void harmonic_walk(int ndata, double m, double psi, Body&& body) {
  double s1, c1;
  sincos(psi, &s1, &c1);
  double sj, cj;
  sincos((double)ndata * psi, &sj, &cj);
  const double am = fabs(m);
  if (m == 0.0 || am < DFMI_BES_TINY || !(am < 1.0e5)) {
    for (int j = ndata; j >= 1; --j) {
      double jm1, j0, jp1;
      if (m == 0.0) {
        jm1 = (j == 1) ? 1.0 : 0.0;
        j0 = jp1 = 0.0;
      } else if (am < DFMI_BES_TINY) {
        jm1 = dfmi_bessel_series(j - 1, m);
        j0 = dfmi_bessel_series(j, m);
        jp1 = dfmi_bessel_series(j + 1, m);
      } else {
        jm1 = j0 = jp1 = __builtin_nan("");
      }
      body(j, jm1, j0, jp1, cj, sj);
      const double cn = fma(cj, c1, sj * s1);
      const double sn = fma(sj, c1, -(cj * s1));
      cj = cn;
      sj = sn;
    }
    return;
  }
  if (dfmi_bessel_use_large(am, ndata + 1)) {
    // runaway descents (|m| >= 64, e.g. ~900): J_0, J_1 asymptotically, then upward
    // (dfmi_math.h), the harmonics visited in ascending order with (cos, sin)(j psi) by
    // rotation upward from (cos, sin)(psi)
    double jm1, j0;
    dfmi_bessel_j01_large(am, &jm1, &j0);
    const double tox = 2.0 / am;
    const double sg = m < 0.0 ? -1.0 : 1.0;  // J_k(-x) = (-1)^k J_k(x)
    double cu = c1, su = s1;                 // (cos, sin)(j psi), j = 1
    for (int j = 1; j <= ndata; ++j) {
      const double jp1 = fma((double)j * tox, j0, -jm1);
      // signs of J_{j-1}, J_j, J_{j+1} at m < 0: (-1)^(j-1), (-1)^j, (-1)^(j+1)
      const double sj0 = (j & 1) ? sg : 1.0, sjm = (j & 1) ? 1.0 : sg;
      body(j, sjm * jm1, sj0 * j0, sjm * jp1, cu, su);
      const double cn = fma(cu, c1, -(su * s1));
      const double sn = fma(su, c1, cu * s1);
      cu = cn;
      su = sn;
      jm1 = j0;
      j0 = jp1;
    }
    return;
  }
  const int M = dfmi_bessel_start(ndata + 1, am);
  int ef = 0;
  const double S = dfmi_bessel_norm(am, M, &ef);
  DfmiBesselWalk w;
  w.init(m, M, S, ef);
  double jp1, j0, jm1;
  for (int k = M; k > ndata; --k) w.step(&jp1, &j0, &jm1);
  for (int j = ndata; j >= 1; --j) {
    w.step(&jp1, &j0, &jm1);
    body(j, jm1, j0, jp1, cj, sj);
    const double cn = fma(cj, c1, sj * s1);     // cos((j-1) psi)
    const double sn = fma(sj, c1, -(cj * s1));  // sin((j-1) psi)
    cj = cn;
    sj = sn;
  }
}

constexpr int kQPre = 4;
template <typename QF, typename = void>
struct QfBes {
  static constexpr bool value = false;
};
template <typename QF>
struct QfBes<QF, std::void_t<decltype(QF::kBes)>> {
  static constexpr bool value = QF::kBes;
};
template <typename QF>
constexpr bool qf_bes() {
  return QfBes<QF>::value;
}

// harmonic_walk handing the body its harmonic's QI as well (body(j, J_{j-1}, J_j, J_{j+1},
// cos j psi, sin j psi, Q_j, I_j)). On the Miller branch (every ordinary m) the QI of
// harmonic j - kQPre is loaded while harmonic j is evaluated, kQPre pairs in registers: the
// walk is otherwise one L2 round trip per harmonic (QI from global memory, ~60 per evaluation
// at ndata 62). The same values in the same operations: the same bits.
// Only lm_chunks_kernel's chunk-size-1 path prefetches (QGlobalT<kQPre>: 196 -> 256 VGPRs, still
// two waves per SIMD); elsewhere the registers cost occupancy or spills (the warm-start chain
// kernel one wave per SIMD, the ladder 50 spilled values, the fused seed + demodulation
// kernel 229), so QGlobal, QRow and QRegs keep kPre = 0 (plain loads).
template <typename QF, typename Body>
DFMI_HDI void harmonic_walk_q(int ndata, double m, double psi, const QF& q, Body&& body) {
  const double am = fabs(m);
  if (QF::kPre == 0 || m == 0.0 || am < DFMI_BES_TINY || !(am < 1.0e5) || dfmi_bessel_use_large(am, ndata + 1)) {
    harmonic_walk(ndata, m, psi, [&](int j, double jm1, double j0, double jp1, double cj, double sj) {
      body(j, jm1, j0, jp1, cj, sj, q.qc(j - 1), q.qs(j - 1));
    });
    return;
  }
  double s1, c1;
  sincos(psi, &s1, &c1);
  double sj, cj;
  sincos((double)ndata * psi, &sj, &cj);
  const int M = dfmi_bessel_start(ndata + 1, am);
  int ef = 0;
  double S;
  if constexpr (qf_bes<QF>()) {
    S = dfmi_bessel_norm_store(am, M, &ef, q.bes, 64, ndata);
    if (ef == 0) {  // no rescale: the stored values are pass 2's, J_k = f_k / S
      const double invS = 1.0 / S;
      const bool neg = m < 0.0;
      auto jv = [&](int k) {
        const double v = q.bes[k * 64] * invS;
        return (neg && (k & 1)) ? -v : v;  // J_n(-x) = (-1)^n J_n(x)
      };
      double bq[kQPre], bs[kQPre];
#pragma unroll
      for (int u = 0; u < kQPre; ++u) {
        const int h = ndata - 1 - u > 0 ? ndata - 1 - u : 0;
        bq[u] = q.qc(h);
        bs[u] = q.qs(h);
      }
      auto one = [&](int j, double qcv, double qsv) {
        body(j, jv(j - 1), jv(j), jv(j + 1), cj, sj, qcv, qsv);
        const double cn = fma(cj, c1, sj * s1);
        const double sn = fma(sj, c1, -(cj * s1));
        cj = cn;
        sj = sn;
      };
      int j = ndata;
      for (; j >= kQPre; j -= kQPre) {
#pragma unroll
        for (int u = 0; u < kQPre; ++u) {
          const double qcv = bq[u], qsv = bs[u];
          const int h = j - 1 - u - kQPre > 0 ? j - 1 - u - kQPre : 0;
          bq[u] = q.qc(h);
          bs[u] = q.qs(h);
          one(j - u, qcv, qsv);
        }
      }
#pragma unroll
      for (int u = 0; u < kQPre; ++u)
        if (u < j) one(j - u, bq[u], bs[u]);
      return;
    }
  } else {
    S = dfmi_bessel_norm(am, M, &ef);
  }
  DfmiBesselWalk w;
  w.init(m, M, S, ef);
  double bq[kQPre], bs[kQPre];  // slot u: harmonic j - u of the block starting at j
#pragma unroll
  for (int u = 0; u < kQPre; ++u) {
    const int h = ndata - 1 - u > 0 ? ndata - 1 - u : 0;
    bq[u] = q.qc(h);
    bs[u] = q.qs(h);
  }
  double jp1, j0, jm1;
  for (int k = M; k > ndata; --k) w.step(&jp1, &j0, &jm1);
  auto one = [&](int j, double qcv, double qsv) {
    w.step(&jp1, &j0, &jm1);
    body(j, jm1, j0, jp1, cj, sj, qcv, qsv);
    const double cn = fma(cj, c1, sj * s1);     // cos((j-1) psi)
    const double sn = fma(sj, c1, -(cj * s1));  // sin((j-1) psi)
    cj = cn;
    sj = sn;
  };
  int j = ndata;
  for (; j >= kQPre; j -= kQPre) {
#pragma unroll
    for (int u = 0; u < kQPre; ++u) {
      const double qcv = bq[u], qsv = bs[u];
      const int h = j - 1 - u - kQPre > 0 ? j - 1 - u - kQPre : 0;  // next block's slot u (clamped)
      bq[u] = q.qc(h);
      bs[u] = q.qs(h);
      one(j - u, qcv, qsv);
    }
  }
#pragma unroll
  for (int u = 0; u < kQPre; ++u)
    if (u < j) one(j - u, bq[u], bs[u]);
}

// QI accessors. qc(h) = Q_{h+1} (cos), qs(h) = I_{h+1} (sin), dc() = the segment mean.
//  QGlobal: component-major qi[c·ld + s] (dfmi_demod's layout; dc lives elsewhere).
//  QRow<STRIDE>: one demodulation row per segment (demod.h qi_row_pos): blocks of
//  16 doubles [cos h0..7 | sin h0..7] per 8 harmonics, dc in a spare slot;
//  STRIDE = 1 for a row in global memory, 65 for a wave's rows transposed into LDS.
//  kPre: QI pairs harmonic_walk_q keeps in flight for the accessor (0: plain loads).
//  BES: harmonic_walk_q may keep the lane's Bessel recurrence values in `bes` (LDS, stride 64:
//  ndata + 2 doubles) and walk once instead of twice.
template <int PRE = 0, bool BES = false>
struct QGlobalT {
  static constexpr int kPre = PRE;
  static constexpr bool kBes = BES;
  const double* __restrict__ p;
  int64_t ld;
  int nd;
  double* bes = nullptr;
  DFMI_HDI double qc(int h) const { return p[(int64_t)h * ld]; }
  DFMI_HDI double qs(int h) const { return p[(int64_t)(nd + h) * ld]; }
};
using QGlobal = QGlobalT<>;

template <int STRIDE>
struct QRow {
  static constexpr int kPre = 0;
  const double* __restrict__ p;
  DFMI_HDI double qc(int h) const { return p[((h >> 3) * 16 + (h & 7)) * STRIDE]; }
  DFMI_HDI double qs(int h) const { return p[((h >> 3) * 16 + 8 + (h & 7)) * STRIDE]; }
  DFMI_HDI double at(int pos) const { return p[pos * STRIDE]; }
};

// QI of one segment held in registers (N harmonics, read once from another accessor):
// the register path's evaluations then index it with compile-time harmonics only.
template <int N>
struct QRegs {
  static constexpr int kPre = 0;
  double c[N], s[N];
  template <typename QF>
  DFMI_HDI void load(const QF& q) {
#pragma unroll
    for (int h = 0; h < N; ++h) {
      c[h] = q.qc(h);
      s[h] = q.qs(h);
    }
  }
  DFMI_HDI double qc(int h) const { return c[h]; }
  DFMI_HDI double qs(int h) const { return s[h]; }
};

template <typename QF>
DFMI_HDI void eval_gen(const QF& q, int nd, const double (&p)[4], Eval& e) {
  const double a = p[0], m = p[1], phi = p[2], psi = p[3];
  double sph, cph;
  sincos(phi, &sph, &cph);
  const bool a_nz = (a != 0.0);
  eval_zero(e);
  harmonic_walk_q(nd, m, psi, q, [&](int j, double Jm1, double J0, double Jp1, double cj, double sj, double qc,
                                     double qs) {
    harmonic_term(e, j, a, a_nz, cph, sph, Jm1, J0, Jp1, cj, sj, qc, qs);
  });
}

// ssqf (fit.py:152-167) on the general path: the ssq part of eval_gen alone, the same
// operations in the same order (harmonic_term's rq, ri and its two fma accumulations over
// the descending harmonic walk), so it equals eval_gen(...).ssq bit for bit.
template <typename QF>
DFMI_HDI double ssq_gen(const QF& q, int nd, const double (&p)[4]) {
  const double a = p[0], m = p[1], phi = p[2], psi = p[3];
  double sph, cph;
  sincos(phi, &sph, &cph);
  double ssq = 0.0;
  harmonic_walk_q(nd, m, psi, q, [&](int j, double, double J0, double, double cj, double sj, double qc, double qs) {
    const double pt = quarter_turn(j, cph, sph);
    const double common = a * pt * J0;
    const double rq = fma(-common, cj, qc);
    const double ri = fma(common, sj, qs);
    ssq = fma(rq, rq, ssq);
    ssq = fma(ri, ri, ssq);
  });
  return ssq;
}

// ---------------------------------------------------------------------------
// Shared LM pieces
// ---------------------------------------------------------------------------

// fit.py:169-206 (msolve): (JtJ + lam diag(JtJ)) dp = Jt r by LU with partial
// pivoting (LAPACK dgesv semantics: first max |pivot|; an exactly-zero pivot
// is a singular matrix -> LinAlgError in numpy -> dp = 0). Fully unrolled, the
// row exchanges are selects: no runtime-indexed array.
DFMI_HDI void damped_solve(const Eval& e, double lam, double (&dp)[4]) {
  double A[4][4] = {{e.a00 + lam * e.a00, e.a01, e.a02, e.a03},
                    {e.a01, e.a11 + lam * e.a11, e.a12, e.a13},
                    {e.a02, e.a12, e.a22 + lam * e.a22, e.a23},
                    {e.a03, e.a13, e.a23, e.a33 + lam * e.a33}};
  double b[4] = {e.g0, e.g1, e.g2, e.g3};
  double invd[4];
  bool singular = false;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    int piv = c;
    double best = fabs(A[c][c]);
#pragma unroll
    for (int r = c + 1; r < 4; ++r) {
      const double v = fabs(A[r][c]);
      if (v > best) {
        best = v;
        piv = r;
      }
    }
#pragma unroll
    for (int r = c + 1; r < 4; ++r) {
      const bool sw = (r == piv);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double t = A[c][k];
        A[c][k] = sw ? A[r][k] : A[c][k];
        A[r][k] = sw ? t : A[r][k];
      }
      const double t = b[c];
      b[c] = sw ? b[r] : b[c];
      b[r] = sw ? t : b[r];
    }
    const double pv = A[c][c];
    singular = singular || (pv == 0.0);
    const double inv = 1.0 / pv;
    invd[c] = inv;
#pragma unroll
    for (int r = c + 1; r < 4; ++r) {
      const double l = A[r][c] * inv;
#pragma unroll
      for (int k = c + 1; k < 4; ++k) A[r][k] = fma(-l, A[c][k], A[r][k]);
      b[r] = fma(-l, b[c], b[r]);
    }
  }
#pragma unroll
  for (int r = 3; r >= 0; --r) {
    double s = b[r];
#pragma unroll
    for (int k = r + 1; k < 4; ++k) s = fma(-A[r][k], dp[k], s);
    dp[r] = s * invd[r];
  }
  if (singular) dp[0] = dp[1] = dp[2] = dp[3] = 0.0;
}

DFMI_HDI double sumsq4(double a, double b, double c, double d) { return fma(a, a, fma(b, b, fma(c, c, d * d))); }

// np.linalg.norm(v) < thr without the square root (thr <= 0: never; the squares
// compare the same numbers up to rounding at the boundary).
DFMI_HDI bool norm_below(double ss, double thr) { return thr > 0.0 && ss < thr * thr; }

// fit.py:208-258 (_run_lma_fit), flattened for SIMT: every pass of the loop does
// ONE damped solve and (unless the step is below min_step_norm) ONE trial
// evaluation for each active lane, whatever its position on the lambda ladder.
// The nested form (iterations x ladder) made a wave execute the union of its lanes'
// ladders at every iteration; here a wave runs max over lanes of the trial count.
// Per lane the sequence of solves, trials and acceptances is exactly the nested
// loop's (lm_descend below: same arithmetic, same bits).
// Ev: trial(p, t) -> ssqf at p; accept(p, t, e) -> coeffs at p from the trial's
// state; solve(e, lambda, dp) -> msolve.
template <typename Ev>
DFMI_HDI double lm_descend_flat(Ev&& ev, double (&p)[4], const LMConst& c) {
  Eval e;
  {
    typename std::decay_t<Ev>::Trial t0;
    ev.trial(p, t0);
    ev.accept(p, t0, e);
  }
  int it = 0, li = 0;
  bool active = c.max_steps > 0 && c.n_lambda > 0;
  while (active) {
    double dp[4];
    ev.solve(e, c.lambdas[li], dp);
    bool accepted = false;
    if (!norm_below(sumsq4(dp[0], dp[1], dp[2], dp[3]), c.min_step_norm)) {
      double pt[4] = {p[0] + dp[0], p[1] + dp[1], p[2] + dp[2], p[3] + dp[3]};
      typename std::decay_t<Ev>::Trial tt;
      const double ssq_try = ev.trial(pt, tt);
      if (ssq_try < e.ssq) {
        accepted = true;
        const double change2 = sumsq4(pt[0] - p[0], pt[1] - p[1], pt[2] - p[2], pt[3] - p[3]);
        p[0] = pt[0];
        p[1] = pt[1];
        p[2] = pt[2];
        p[3] = pt[3];
        const double best_ssq = ssq_try;
        ++it;
        li = 0;
        // coeffs(ndata, data, parm) at the accepted point (fit.py:251): its ssq is the trial's
        // (both evaluators reuse the trial's sum), so the convergence test (fit.py:254-256) is
        // known before it; a point the descent stops at needs only that ssq, not J^T J / J^T r
        if (((ev.ssq_of(tt) - best_ssq) < c.conv_improve && norm_below(change2, c.conv_param_change)) ||
            it >= c.max_steps) {
          e.ssq = ev.ssq_of(tt);
          active = false;
        } else {
          ev.accept(p, tt, e);
        }
      }
    }
    if (!accepted && ++li >= c.n_lambda) active = false;  // no lambda improved: fit.py:246-247
  }
  return e.ssq;
}

// Evaluators for the descents: trial(p, t) = ssqf at p, accept(p, t, e) = coeffs at an
// accepted p, solve = msolve. General path (GenSplitEval one lane per fit, FullGenEval on
// the lambda ladder): the literal evaluation + the pivoting 4x4 solve; register path
// (SplitEval): the structured evaluation, block-diagonal solve.
// General path, one full literal evaluation per trial: the trial state is the whole Eval,
// so an accepted trial needs no second evaluation. The lambda-ladder descent takes this
// one (its 8 lanes evaluate 8 rungs at once and accept by shuffling the taken rung's state):
// with GenSplitEval there the seed of a phi = 1.3, psi = 0.4 record took 17.5 ms against
// 9.2 ms (tests/test_gpu_numerics.py::test_seed_wave_ladder_equals_one_lane_general_fit,
// r04c), every accepted iteration paying a second evaluation.
template <typename QF>
struct FullGenEval {
  const QF& q;
  int nd;
  struct Trial {
    Eval e;
  };
  DFMI_HDI double trial(const double (&p)[4], Trial& t) {
    eval_gen(q, nd, p, t.e);
    return t.e.ssq;
  }
  DFMI_HDI void accept(const double (&)[4], const Trial& t, Eval& e) { e = t.e; }
  DFMI_HDI void solve(const Eval& e, double lam, double (&dp)[4]) { damped_solve(e, lam, dp); }
  DFMI_HDI static double ssq_of(const Trial& t) { return t.e.ssq; }
};

// General path, split like the register path: a trial evaluates ssqf only (ssq_gen), the
// literal coeffs (eval_gen: J^T J, J^T r) runs at accepted points only; same bits as
// a full literal evaluation per trial (ssq_gen == eval_gen().ssq), about half the work per rejected rung — the rungs a
// descent walks at the noise floor or far from the minimum (the record pipeline's seed).
template <typename QF>
struct GenSplitEval {
  const QF& q;
  int nd;
  struct Trial {
    double ssq;
  };
  DFMI_HDI double trial(const double (&p)[4], Trial& t) {
    t.ssq = ssq_gen(q, nd, p);
    return t.ssq;
  }
  DFMI_HDI void accept(const double (&p)[4], const Trial&, Eval& e) { eval_gen(q, nd, p, e); }
  DFMI_HDI void solve(const Eval& e, double lam, double (&dp)[4]) { damped_solve(e, lam, dp); }
  DFMI_HDI static double ssq_of(const Trial& t) { return t.ssq; }
};

template <int NDMAX, typename QF>
struct SplitEval {  // NDMAX: a register-path variant tag (nd_cap / nd_exact)
  const QF& q;
  int nd;
  const DfmiTrigK& k;
  using Trial = TrialReg<NDMAX>;
  DFMI_HDI double trial(const double (&p)[4], Trial& t) { return eval_reg_trial<NDMAX>(q, nd, p, t, k); }
  DFMI_HDI void accept(const double (&p)[4], const Trial& t, Eval& e) { eval_reg_accept<NDMAX>(q, nd, p, t, e); }
  DFMI_HDI void solve(const Eval& e, double lam, double (&dp)[4]) { damped_solve_block(e, lam, dp); }
  DFMI_HDI static double ssq_of(const Trial& t) { return t.ssq; }
};

// ---------------------------------------------------------------------------
// Many-harmonic path (ndata > 16): the register path's structured evaluation over a lean
// Miller walk.
//
// The general path above spends ~71k VALU instructions per wave of 64 fits at ndata 62
// (config-2 QI; profiles/r06/lm_general_pmc_before.txt): each harmonic of a full evaluation
// is ~85 instructions (the literal per-residual Jacobian, quarter_turn selects on a runtime
// j, 64-bit QI addressing) and each step of the two Miller passes ~10 more (the per-step
// overflow test and the rescale bookkeeping of dfmi_math.h). A wave issues those back to back
// (fp64 chains are issue-bound, dfmi_math.h dfmi_sincos_k), so the LM's time is its
// instruction count. Here:
//  * the two Miller passes without per-step tests where no rescale can happen: |f_{k-1}| <=
//    (2k/x + 1) |f_k|, so M log2(2M/x + 1) < 590 keeps every f below 2^600 (the walk's rescale
//    threshold) and the values are bit for bit those of the checked walk (same fma sequence);
//    otherwise (tiny / huge / negative m, or a bound that does not hold) the checked walk of
//    harmonic_walk;
//  * harmonics in blocks of four with j = 4b - u, so cos(phi + j pi/2) is a signed (a cos phi,
//    a sin phi) without a select;
//  * the closed-form J^T J / J^T r of eval_reg_accept (psi column orthogonal: block-diagonal
//    J^T J, damped_solve_block) and ssqf-only trials as on the register path;
//  * QI through QCol: a uniform column base plus a 32-bit per-lane offset (no 64-bit address
//    arithmetic per load), the next block's four QI pairs loaded while this block is evaluated.
// Not bit-identical to the literal general path (lm_general = 1 keeps that one); parity with
// the reference is gated at full scale (tests/test_gpu_full_scale.py ndata 16..62,
// tests/test_gpu_quickstart.py).
// ---------------------------------------------------------------------------
constexpr int kWideNd = 1 << 9;       // NDMAX tag of the many-harmonic path
constexpr int kWideNdF = kWideNd | 1;  // the same with one walk per trial (WideEval<QF, true>)
constexpr bool wide_nd(int ndmax) { return (ndmax & ~1) == kWideNd; }

// Component-major QI with the column base uniform across the wave (qi, harmonic h) and the
// segment index per lane.
struct QCol {
  static constexpr int kPre = 0;
  const double* __restrict__ base;
  uint32_t off;
  int64_t ld;
  int nd;
  DFMI_HDI double qc(int h) const { return (base + (int64_t)h * ld)[off]; }
  DFMI_HDI double qs(int h) const { return (base + (int64_t)(nd + h) * ld)[off]; }
};

// The lane's own QI staged in LDS by lm_chunks_kernel (column c of the lane at p[c * 64]): every
// evaluation of a fit reads each value again, and from L2 / the MALL the wave waited on those
// loads for half its lifetime (profiles/r06/lm_general_pmc_after.txt).
struct QLds {
  static constexpr int kPre = 0;
  const double* p;
  int nd;
  DFMI_HDI double qc(int h) const { return p[h * 64]; }
  DFMI_HDI double qs(int h) const { return p[(nd + h) * 64]; }
};

// Harmonics j = nd .. 1 in descending order: body(j, J_{j-1}, J_j, J_{j+1}, cos j psi, sin j psi,
// Q_j, I_j). (c1, s1) = (cos, sin) psi, (cn, sn) = (cos, sin)(nd psi).
template <typename QF, typename Body>
DFMI_HDI void wide_walk(const QF& q, int nd, double m, double psi, double c1, double s1, double cn, double sn,
                        Body&& body) {
  const int M = dfmi_bessel_start(nd + 1, m);
  const double tox = 2.0 / m;
  const bool fast = m > 0.0 && m >= DFMI_BES_TINY && m < 1.0e5 && !dfmi_bessel_use_large(m, nd + 1) &&
                    (float)M * log2f((float)fma((double)M, tox, 1.0)) < (float)(DFMI_BES_BIG_EXP - 10);
  if (!fast) {
    harmonic_walk(nd, m, psi, [&](int j, double jm1, double j0, double jp1, double cj, double sj) {
      body(j, jm1, j0, jp1, cj, sj, q.qc(j - 1), q.qs(j - 1));
    });
    return;
  }
  // the QI of the first two blocks of four, issued before the Miller passes (which need none)
  // so that their latency hides behind them; each later block is loaded two blocks (8
  // harmonics) ahead of its use. (Four blocks ahead, 64 more VGPRs, took the kernel past 256
  // VGPRs into scratch: 0.29 ms at ndata 62 against 0.22, r06e.)
  const int top = nd & 3, nb = nd >> 2;
  double bq[2][4], bs[2][4];  // ring of two blocks: slot i holds block nb - i
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int blk = nb - i;
      const int h = blk >= 1 ? 4 * blk - 1 - u : 0;
      bq[i][u] = q.qc(h);
      bs[i][u] = q.qs(h);
    }
  // pass 1: S = f_0 + 2 sum f_2k (M even; dfmi_bessel_norm without its rescale test)
  double fp1 = 0.0, f = 1.0, S = 2.0;
  double kd = (double)M;
  for (int k = M; k > 2; k -= 2) {
    double fm1 = fma(kd * tox, f, -fp1);
    fp1 = f;
    f = fm1;
    kd -= 1.0;
    fm1 = fma(kd * tox, f, -fp1);
    fp1 = f;
    f = fm1;
    kd -= 1.0;
    S += 2.0 * f;  // f_{k-2}, an even order > 0
  }
  {
    double fm1 = fma(kd * tox, f, -fp1);  // f_1
    fp1 = f;
    f = fm1;
    kd -= 1.0;
    fm1 = fma(kd * tox, f, -fp1);  // f_0
    S += fm1;
  }
  const double invS = 1.0 / S;
  // pass 2: down to f_{nd+1}, then one step per harmonic
  fp1 = 0.0;
  f = 1.0;
  kd = (double)M;
  for (int k = M; k > nd + 1; --k) {
    const double fm1 = fma(kd * tox, f, -fp1);
    fp1 = f;
    f = fm1;
    kd -= 1.0;
  }
  // f = f_{nd+1}, fp1 = f_{nd+2}, kd = nd + 1
  double Jp1 = f * invS;
  {
    const double fm1 = fma(kd * tox, f, -fp1);  // f_nd
    fp1 = f;
    f = fm1;
    kd -= 1.0;
  }
  double J0 = f * invS;
  double cj = cn, sj = sn;
  auto one = [&](int j, double Q, double I) {
    const double fm1 = fma(kd * tox, f, -fp1);  // f_{j-1}
    fp1 = f;
    f = fm1;
    kd -= 1.0;
    const double Jm1 = fm1 * invS;
    body(j, Jm1, J0, Jp1, cj, sj, Q, I);
    Jp1 = J0;
    J0 = Jm1;
    const double c2 = fma(cj, c1, sj * s1);     // cos((j-1) psi)
    const double s2 = fma(sj, c1, -(cj * s1));  // sin((j-1) psi)
    cj = c2;
    sj = s2;
  };
  for (int u = 0; u < top; ++u) one(nd - u, q.qc(nd - 1 - u), q.qs(nd - 1 - u));
  // blocks of four from a multiple of four (j = 4 blk - u: j & 3 known at compile time), each
  // block's QI loaded two blocks (8 harmonics) ahead of its use
  auto block = [&](int slot, int blk) {
    double cq[4], cs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      cq[u] = bq[slot][u];
      cs[u] = bs[slot][u];
      const int h = blk - 2 >= 1 ? 4 * (blk - 2) - 1 - u : 0;  // two blocks ahead (clamped)
      bq[slot][u] = q.qc(h);
      bs[slot][u] = q.qs(h);
    }
    const int jb = blk << 2;
#pragma unroll
    for (int u = 0; u < 4; ++u) one(jb - u, cq[u], cs[u]);
  };
  int b = nb;
  for (; b >= 2; b -= 2) {
    block(0, b);
    block(1, b - 1);
  }
  if (b == 1) block(0, 1);
}

struct WideTrial {
  double ssq, cph, sph, c1, s1, cn, sn;
};

// ssqf (fit.py:152-167) at p on the many-harmonic path; keeps the point's trig in t.
template <typename QF>
DFMI_HDI double wide_trial(const QF& q, int nd, const double (&p)[4], WideTrial& t, const DfmiTrigK& k) {
  dfmi_sincos_auto(p[2], k, &t.sph, &t.cph);
  dfmi_sincos_auto(p[3], k, &t.s1, &t.c1);
  dfmi_sincos_auto((double)nd * p[3], k, &t.sn, &t.cn);
  const double ac = p[0] * t.cph, as = p[0] * t.sph;
  double so = 0.0, se = 0.0;
  wide_walk(q, nd, p[1], p[3], t.c1, t.s1, t.cn, t.sn,
            [&](int j, double, double J0, double, double cj, double sj, double Q, double I) {
              const double c = quarter_turn(j, ac, as) * J0;  // a cos(phi + j pi/2) J_j
              const double rq = fma(-c, cj, Q);
              const double ri = fma(c, sj, I);
              if (j & 1) {
                so = fma(rq, rq, so);
                so = fma(ri, ri, so);
              } else {
                se = fma(rq, rq, se);
                se = fma(ri, ri, se);
              }
            });
  t.ssq = so + se;
  return t.ssq;
}

// coeffs (fit.py:68-150) at an accepted trial point: eval_reg_accept's closed form over the
// many-harmonic walk; e.ssq is the trial's.
template <typename QF>
DFMI_HDI void wide_accept(const QF& q, int nd, const double (&p)[4], const WideTrial& t, Eval& e) {
  const double a = p[0];
  const double ac = a * t.cph, as = a * t.sph;
  const double cph0 = (a != 0.0) ? t.cph : 0.0, sph0 = (a != 0.0) ? t.sph : 0.0;
  double a00 = 0.0, a01 = 0.0, a02 = 0.0, a11 = 0.0, a12 = 0.0, a22 = 0.0, a33 = 0.0;
  double g0 = 0.0, g1 = 0.0, g2 = 0.0, g3 = 0.0;
  wide_walk(q, nd, p[1], p[3], t.c1, t.s1, t.cn, t.sn,
            [&](int j, double Jm1, double Jj, double Jp1, double cj, double sj, double Q, double I) {
              const double aP = quarter_turn(j, ac, as), aD = quarter_turn(j + 1, ac, as);
              const double c = aP * Jj;
              const double u0 = quarter_turn(j, cph0, sph0) * Jj;
              const double u1 = aP * (0.5 * (Jm1 - Jp1));
              const double u2 = aD * Jj;
              const double rq = fma(-c, cj, Q);
              const double ri = fma(c, sj, I);
              const double A = fma(cj, rq, -(sj * ri));
              const double B = fma(sj, rq, cj * ri);
              // cos^2 + sin^2 of the rotation taken as 1 (it is to ~1e-14 after 62 rotations):
              // J^T J moves by that much relative, the step direction with it, ssq not at all
              a00 = fma(u0, u0, a00);
              a01 = fma(u0, u1, a01);
              a02 = fma(u0, u2, a02);
              a11 = fma(u1, u1, a11);
              a12 = fma(u1, u2, a12);
              a22 = fma(u2, u2, a22);
              const double jc = (double)j * c;
              a33 = fma(jc, jc, a33);
              g0 = fma(u0, A, g0);
              g1 = fma(u1, A, g1);
              g2 = fma(u2, A, g2);
              g3 = fma(-jc, B, g3);
            });
  e = Eval{t.ssq, a00, a01, a02, 0.0, a11, a12, 0.0, a22, 0.0, a33, g0, g1, g2, g3};
}

// ssqf and coeffs at p in ONE walk (WideEval<QF, true>): the bodies of wide_trial and
// wide_accept together, the same operations on the same walk values, so the same bits as a
// trial followed by its accept. The LM runs SIMT: a wave pays the accept's walk on every pass
// where one of its 64 lanes accepts (nearly every pass but the last few), so a trial that
// carries the coeffs costs ~the accept alone where the split form costs trial + accept.
struct WideFull {
  Eval e;
};

template <typename QF>
DFMI_HDI double wide_full(const QF& q, int nd, const double (&p)[4], Eval& e, const DfmiTrigK& k) {
  double sph, cph, s1, c1, sn, cn;
  dfmi_sincos_auto(p[2], k, &sph, &cph);
  dfmi_sincos_auto(p[3], k, &s1, &c1);
  dfmi_sincos_auto((double)nd * p[3], k, &sn, &cn);
  const double a = p[0];
  const double ac = a * cph, as = a * sph;
  const double cph0 = (a != 0.0) ? cph : 0.0, sph0 = (a != 0.0) ? sph : 0.0;
  double so = 0.0, se = 0.0;
  double a00 = 0.0, a01 = 0.0, a02 = 0.0, a11 = 0.0, a12 = 0.0, a22 = 0.0, a33 = 0.0;
  double g0 = 0.0, g1 = 0.0, g2 = 0.0, g3 = 0.0;
  wide_walk(q, nd, p[1], p[3], c1, s1, cn, sn,
            [&](int j, double Jm1, double Jj, double Jp1, double cj, double sj, double Q, double I) {
              const double aP = quarter_turn(j, ac, as), aD = quarter_turn(j + 1, ac, as);
              const double c = aP * Jj;
              const double rq = fma(-c, cj, Q);
              const double ri = fma(c, sj, I);
              if (j & 1) {
                so = fma(rq, rq, so);
                so = fma(ri, ri, so);
              } else {
                se = fma(rq, rq, se);
                se = fma(ri, ri, se);
              }
              const double u0 = quarter_turn(j, cph0, sph0) * Jj;
              const double u1 = aP * (0.5 * (Jm1 - Jp1));
              const double u2 = aD * Jj;
              const double A = fma(cj, rq, -(sj * ri));
              const double B = fma(sj, rq, cj * ri);
              a00 = fma(u0, u0, a00);
              a01 = fma(u0, u1, a01);
              a02 = fma(u0, u2, a02);
              a11 = fma(u1, u1, a11);
              a12 = fma(u1, u2, a12);
              a22 = fma(u2, u2, a22);
              const double jc = (double)j * c;
              a33 = fma(jc, jc, a33);
              g0 = fma(u0, A, g0);
              g1 = fma(u1, A, g1);
              g2 = fma(u2, A, g2);
              g3 = fma(-jc, B, g3);
            });
  e = Eval{so + se, a00, a01, a02, 0.0, a11, a12, 0.0, a22, 0.0, a33, g0, g1, g2, g3};
  return e.ssq;
}

template <typename QF, bool FUSED = false>
struct WideEval {
  const QF& q;
  int nd;
  const DfmiTrigK& k;
  using Trial = WideTrial;
  DFMI_HDI double trial(const double (&p)[4], Trial& t) { return wide_trial(q, nd, p, t, k); }
  DFMI_HDI void accept(const double (&p)[4], const Trial& t, Eval& e) { wide_accept(q, nd, p, t, e); }
  DFMI_HDI void solve(const Eval& e, double lam, double (&dp)[4]) { damped_solve_block(e, lam, dp); }
  DFMI_HDI static double ssq_of(const Trial& t) { return t.ssq; }
};

template <typename QF>
struct WideEval<QF, true> {
  const QF& q;
  int nd;
  const DfmiTrigK& k;
  using Trial = WideFull;
  DFMI_HDI double trial(const double (&p)[4], Trial& t) { return wide_full(q, nd, p, t.e, k); }
  DFMI_HDI void accept(const double (&)[4], const Trial& t, Eval& e) { e = t.e; }
  DFMI_HDI void solve(const Eval& e, double lam, double (&dp)[4]) { damped_solve_block(e, lam, dp); }
  DFMI_HDI static double ssq_of(const Trial& t) { return t.e.ssq; }
};

// ---------------------------------------------------------------------------
// Many harmonics, P lanes per segment (lm_split_kernel). A wave fits 64 / P segments; lane r
// of a segment's group walks a contiguous share of the harmonics (r = 0 the top nd / P), its
// own Miller recurrence down to that share (pass 1 in full on every lane) and rotation start
// (cos, sin)(hi psi); the harmonic sums are partial per lane and reduced over the group by an
// xor butterfly within the quad (DPP): every lane of the group ends with the same bits, so the
// group takes the LM's decisions together (one control flow per segment). QI are staged in
// LDS by the kernel: 64 / P segments x 2 ndata doubles per wave (31 KB at ndata 62, P = 2).
// ---------------------------------------------------------------------------
template <int S>
struct QLdsG {  // QI of one segment in a wave's LDS tile [component][S segments]
  static constexpr int kPre = 0;
  const double* p;
  int nd;
  DFMI_HDI double qc(int h) const { return p[h * S]; }
  DFMI_HDI double qs(int h) const { return p[(nd + h) * S]; }
};

// sum of v over the P lanes of a group (P = 1, 2, 4, 8: lanes r = lane % P), the same bits on
// every lane of the group (each butterfly level adds two commuted operands)
template <int P>
__device__ __forceinline__ double group_sum(double v) {
  if constexpr (P >= 2) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = (int)b, hi = (int)(b >> 32);
    const int lo1 = __builtin_amdgcn_update_dpp(0, lo, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    const int hi1 = __builtin_amdgcn_update_dpp(0, hi, 0xB1, 0xF, 0xF, false);
    v += __builtin_bit_cast(double, ((long long)hi1 << 32) | (unsigned)lo1);
  }
  if constexpr (P >= 4) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = (int)b, hi = (int)(b >> 32);
    const int lo2 = __builtin_amdgcn_update_dpp(0, lo, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    const int hi2 = __builtin_amdgcn_update_dpp(0, hi, 0x4E, 0xF, 0xF, false);
    v += __builtin_bit_cast(double, ((long long)hi2 << 32) | (unsigned)lo2);
  }
  if constexpr (P >= 8) {  // the two quads of a half-row: lane i <- 7 - i (the other quad's sum)
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = (int)b, hi = (int)(b >> 32);
    const int lo3 = __builtin_amdgcn_update_dpp(0, lo, 0x141, 0xF, 0xF, false);  // row_half_mirror
    const int hi3 = __builtin_amdgcn_update_dpp(0, hi, 0x141, 0xF, 0xF, false);
    v += __builtin_bit_cast(double, ((long long)hi3 << 32) | (unsigned)lo3);
  }
  static_assert(P == 1 || P == 2 || P == 4 || P == 8, "P");
  return v;
}

// wide_walk over lane r's share of the harmonics: j = hi .. lo with hi = nd - r ceil(nd / P).
template <int P, typename QF, typename Body>
__device__ __forceinline__ void wide_walk_part(const QF& q, int nd, double m, double psi, double c1, double s1,
                                               const DfmiTrigK& tk, int r, Body&& body) {
  const int len = (nd + P - 1) / P;
  const int hi = nd - r * len;
  const int lo = hi - len + 1 > 1 ? hi - len + 1 : 1;
  const int M = dfmi_bessel_start(nd + 1, m);
  const double tox = 2.0 / m;
  const bool fast = m > 0.0 && m >= DFMI_BES_TINY && m < 1.0e5 && !dfmi_bessel_use_large(m, nd + 1) &&
                    (float)M * log2f((float)fma((double)M, tox, 1.0)) < (float)(DFMI_BES_BIG_EXP - 10);
  if (!fast) {  // the checked walk of every harmonic, this lane's share accumulated
    harmonic_walk(nd, m, psi, [&](int j, double jm1, double j0, double jp1, double cj, double sj) {
      if (j <= hi && j >= lo) body(j, jm1, j0, jp1, cj, sj, q.qc(j - 1), q.qs(j - 1));
    });
    return;
  }
  if (hi < 1) return;  // no share (nd < P)
  double sn, cn;
  dfmi_sincos_auto((double)hi * psi, tk, &sn, &cn);
  double nq = q.qc(hi - 1), ni = q.qs(hi - 1);
  // pass 1 (as wide_walk)
  double fp1 = 0.0, f = 1.0, S = 2.0;
  double kd = (double)M;
  for (int k = M; k > 2; k -= 2) {
    double fm1 = fma(kd * tox, f, -fp1);
    fp1 = f;
    f = fm1;
    kd -= 1.0;
    fm1 = fma(kd * tox, f, -fp1);
    fp1 = f;
    f = fm1;
    kd -= 1.0;
    S += 2.0 * f;
  }
  {
    double fm1 = fma(kd * tox, f, -fp1);
    fp1 = f;
    f = fm1;
    kd -= 1.0;
    fm1 = fma(kd * tox, f, -fp1);
    S += fm1;
  }
  const double invS = 1.0 / S;
  // pass 2 down to this lane's share (a per-lane trip count)
  fp1 = 0.0;
  f = 1.0;
  kd = (double)M;
  for (int k = M; k > hi + 1; --k) {
    const double fm1 = fma(kd * tox, f, -fp1);
    fp1 = f;
    f = fm1;
    kd -= 1.0;
  }
  double Jp1 = f * invS;
  {
    const double fm1 = fma(kd * tox, f, -fp1);  // f_hi
    fp1 = f;
    f = fm1;
    kd -= 1.0;
  }
  double J0 = f * invS;
  double cj = cn, sj = sn;
  for (int j = hi; j >= lo; --j) {
    const double Q = nq, I = ni;
    const int h = j > lo ? j - 2 : j - 1;  // the next harmonic's QI (LDS)
    nq = q.qc(h);
    ni = q.qs(h);
    const double fm1 = fma(kd * tox, f, -fp1);  // f_{j-1}
    fp1 = f;
    f = fm1;
    kd -= 1.0;
    const double Jm1 = fm1 * invS;
    body(j, Jm1, J0, Jp1, cj, sj, Q, I);
    Jp1 = J0;
    J0 = Jm1;
    const double c2 = fma(cj, c1, sj * s1);
    const double s2 = fma(sj, c1, -(cj * s1));
    cj = c2;
    sj = s2;
  }
}

// wide_walk_part in ONE Miller pass (the seed's evaluator): the P lanes of a rung walk the same
// recurrence (the same trial m), so each stores every f_k it forms in the rung's LDS row `fb`
// while summing the normalisation as pass 1 does, then reads back its share's f_{lo-1} ..
// f_{hi+1}: the recurrence runs M steps per evaluation instead of M + (M - lo), with the same
// values (bit for bit wide_walk_part's J). kFbMax bounds M where the lean walk applies
// (M log2(2M/m + 1) < 590 with M >= 1.1 m: M < 351); beyond, wide_walk_part.
constexpr int kFbMax = 356;
template <int P, typename QF, typename Body>
__device__ __forceinline__ void wide_walk_share(const QF& q, int nd, double m, double psi, double c1, double s1,
                                                const DfmiTrigK& tk, int r, double* fb, Body&& body) {
  const int len = (nd + P - 1) / P;
  const int hi = nd - r * len;
  const int lo = hi - len + 1 > 1 ? hi - len + 1 : 1;
  const int M = dfmi_bessel_start(nd + 1, m);
  const double tox = 2.0 / m;
  const bool fast = m > 0.0 && m >= DFMI_BES_TINY && m < 1.0e5 && !dfmi_bessel_use_large(m, nd + 1) &&
                    (float)M * log2f((float)fma((double)M, tox, 1.0)) < (float)(DFMI_BES_BIG_EXP - 10) &&
                    M + 2 <= kFbMax;
  if (!fast) {
    wide_walk_part<P>(q, nd, m, psi, c1, s1, tk, r, body);
    return;
  }
  double fp1 = 0.0, f = 1.0, S = 2.0;
  double kd = (double)M;
  fb[M + 1] = 0.0;
  fb[M] = 1.0;
  for (int k = M; k > 2; k -= 2) {
    double fm1 = fma(kd * tox, f, -fp1);
    fb[k - 1] = fm1;
    fp1 = f;
    f = fm1;
    kd -= 1.0;
    fm1 = fma(kd * tox, f, -fp1);
    fb[k - 2] = fm1;
    fp1 = f;
    f = fm1;
    kd -= 1.0;
    S += 2.0 * f;
  }
  {
    double fm1 = fma(kd * tox, f, -fp1);  // f_1
    fb[1] = fm1;
    fp1 = f;
    f = fm1;
    kd -= 1.0;
    fm1 = fma(kd * tox, f, -fp1);  // f_0
    fb[0] = fm1;
    S += fm1;
  }
  if (hi < 1) return;  // no share (nd < P)
  const double invS = 1.0 / S;
  double sn, cn;
  dfmi_sincos_auto((double)hi * psi, tk, &sn, &cn);
  double Jp1 = fb[hi + 1] * invS;
  double J0 = fb[hi] * invS;
  double cj = cn, sj = sn;
  for (int j = hi; j >= lo; --j) {
    const double Jm1 = fb[j - 1] * invS;
    body(j, Jm1, J0, Jp1, cj, sj, q.qc(j - 1), q.qs(j - 1));
    Jp1 = J0;
    J0 = Jm1;
    const double c2 = fma(cj, c1, sj * s1);
    const double s2 = fma(sj, c1, -(cj * s1));
    cj = c2;
    sj = s2;
  }
}

// The many-harmonic seed's evaluator (FLAT 3: one record's buffer 0 fitted by a whole wave, 8
// rungs x P = 8 shares): wide_full's sums over this lane's share of the harmonics, reduced over
// the P lanes; a trial carries the coeffs (the ladder shuffles the taken rung's Eval, so an
// accepted trial needs no second walk). A lane's walk is the Miller passes + its share: at
// ndata 62 ~1/3 of one lane's full walk. Not bit-identical to WideEval (the sums' order).
template <int P, typename QF>
struct PartFullEval {
  const QF& q;
  int nd;
  const DfmiTrigK& k;
  int r;  // this lane's share
  using Trial = WideFull;
  __device__ __forceinline__ double trial(const double (&p)[4], Trial& t) {
    double sph, cph, s1, c1;
    dfmi_sincos_auto(p[2], k, &sph, &cph);
    dfmi_sincos_auto(p[3], k, &s1, &c1);
    const double a = p[0];
    const double ac = a * cph, as = a * sph;
    const double cph0 = (a != 0.0) ? cph : 0.0, sph0 = (a != 0.0) ? sph : 0.0;
    double ss = 0.0, a00 = 0.0, a01 = 0.0, a02 = 0.0, a11 = 0.0, a12 = 0.0, a22 = 0.0, a33 = 0.0;
    double g0 = 0.0, g1 = 0.0, g2 = 0.0, g3 = 0.0;
    // the rung's LDS row for the one-pass walk (64 / P rungs of P lanes: the whole wave)
    __shared__ double fbuf[64 / P][kFbMax];
    double* fb = fbuf[__lane_id() / P];
    wide_walk_share<P>(q, nd, p[1], p[3], c1, s1, k, r, fb,
                      [&](int j, double Jm1, double Jj, double Jp1, double cj, double sj, double Q, double I) {
                        const double aP = quarter_turn(j, ac, as), aD = quarter_turn(j + 1, ac, as);
                        const double c = aP * Jj;
                        const double rq = fma(-c, cj, Q);
                        const double ri = fma(c, sj, I);
                        ss = fma(rq, rq, ss);
                        ss = fma(ri, ri, ss);
                        const double u0 = quarter_turn(j, cph0, sph0) * Jj;
                        const double u1 = aP * (0.5 * (Jm1 - Jp1));
                        const double u2 = aD * Jj;
                        const double A = fma(cj, rq, -(sj * ri));
                        const double B = fma(sj, rq, cj * ri);
                        a00 = fma(u0, u0, a00);
                        a01 = fma(u0, u1, a01);
                        a02 = fma(u0, u2, a02);
                        a11 = fma(u1, u1, a11);
                        a12 = fma(u1, u2, a12);
                        a22 = fma(u2, u2, a22);
                        const double jc = (double)j * c;
                        a33 = fma(jc, jc, a33);
                        g0 = fma(u0, A, g0);
                        g1 = fma(u1, A, g1);
                        g2 = fma(u2, A, g2);
                        g3 = fma(-jc, B, g3);
                      });
    t.e = Eval{group_sum<P>(ss), group_sum<P>(a00), group_sum<P>(a01), group_sum<P>(a02), 0.0, group_sum<P>(a11),
               group_sum<P>(a12), 0.0, group_sum<P>(a22), 0.0, group_sum<P>(a33), group_sum<P>(g0),
               group_sum<P>(g1), group_sum<P>(g2), group_sum<P>(g3)};
    return t.e.ssq;
  }
  __device__ __forceinline__ void accept(const double (&)[4], const Trial& t, Eval& e) { e = t.e; }
  __device__ __forceinline__ void solve(const Eval& e, double lam, double (&dp)[4]) { damped_solve_block(e, lam, dp); }
  __device__ __forceinline__ static double ssq_of(const Trial& t) { return t.e.ssq; }
};

template <int P, typename QF>
struct PartEval {
  const QF& q;
  int nd;
  const DfmiTrigK& k;
  int r;  // this lane's place in its segment's group
  using Trial = WideTrial;
  __device__ __forceinline__ double trial(const double (&p)[4], Trial& t) {
    dfmi_sincos_auto(p[2], k, &t.sph, &t.cph);
    dfmi_sincos_auto(p[3], k, &t.s1, &t.c1);
    const double ac = p[0] * t.cph, as = p[0] * t.sph;
    double so = 0.0, se = 0.0;
    wide_walk_part<P>(q, nd, p[1], p[3], t.c1, t.s1, k, r,
                      [&](int j, double, double J0, double, double cj, double sj, double Q, double I) {
                        const double c = quarter_turn(j, ac, as) * J0;
                        const double rq = fma(-c, cj, Q);
                        const double ri = fma(c, sj, I);
                        so = fma(rq, rq, so);
                        se = fma(ri, ri, se);
                      });
    t.ssq = group_sum<P>(so + se);
    return t.ssq;
  }
  __device__ __forceinline__ void accept(const double (&p)[4], const Trial& t, Eval& e) {
    const double a = p[0];
    const double ac = a * t.cph, as = a * t.sph;
    const double cph0 = (a != 0.0) ? t.cph : 0.0, sph0 = (a != 0.0) ? t.sph : 0.0;
    double a00 = 0.0, a01 = 0.0, a02 = 0.0, a11 = 0.0, a12 = 0.0, a22 = 0.0, a33 = 0.0;
    double g0 = 0.0, g1 = 0.0, g2 = 0.0, g3 = 0.0;
    wide_walk_part<P>(q, nd, p[1], p[3], t.c1, t.s1, k, r,
                      [&](int j, double Jm1, double Jj, double Jp1, double cj, double sj, double Q, double I) {
                        const double aP = quarter_turn(j, ac, as), aD = quarter_turn(j + 1, ac, as);
                        const double c = aP * Jj;
                        const double u0 = quarter_turn(j, cph0, sph0) * Jj;
                        const double u1 = aP * (0.5 * (Jm1 - Jp1));
                        const double u2 = aD * Jj;
                        const double rq = fma(-c, cj, Q);
                        const double ri = fma(c, sj, I);
                        const double A = fma(cj, rq, -(sj * ri));
                        const double B = fma(sj, rq, cj * ri);
                        const double w = fma(cj, cj, sj * sj);
                        const double v0 = u0 * w, v1 = u1 * w, v2 = u2 * w;
                        a00 = fma(v0, u0, a00);
                        a01 = fma(v0, u1, a01);
                        a02 = fma(v0, u2, a02);
                        a11 = fma(v1, u1, a11);
                        a12 = fma(v1, u2, a12);
                        a22 = fma(v2, u2, a22);
                        const double jc = (double)j * c;
                        a33 = fma(jc * w, jc, a33);
                        g0 = fma(u0, A, g0);
                        g1 = fma(u1, A, g1);
                        g2 = fma(u2, A, g2);
                        g3 = fma(-jc, B, g3);
                      });
    e = Eval{t.ssq, group_sum<P>(a00), group_sum<P>(a01), group_sum<P>(a02), 0.0, group_sum<P>(a11),
             group_sum<P>(a12), 0.0, group_sum<P>(a22), 0.0, group_sum<P>(a33), group_sum<P>(g0), group_sum<P>(g1),
             group_sum<P>(g2), group_sum<P>(g3)};
  }
  __device__ __forceinline__ void solve(const Eval& e, double lam, double (&dp)[4]) { damped_solve_block(e, lam, dp); }
  __device__ __forceinline__ static double ssq_of(const Trial& t) { return t.ssq; }
};

// fit.py:208-258 (_run_lma_fit), nested form (one lane at a time: the host build's
// check that the flattened descent takes the same path). p in/out; returns ssq0 at
// the final p.
template <typename Ev>
DFMI_HDI double lm_descend(Ev&& ev, double (&p)[4], const LMConst& c) {
  Eval e;
  {
    typename std::decay_t<Ev>::Trial t0;
    ev.trial(p, t0);
    ev.accept(p, t0, e);
  }
  for (int it = 0; it < c.max_steps; ++it) {
    const double po0 = p[0], po1 = p[1], po2 = p[2], po3 = p[3];
    bool found = false;
    double pt[4];
    typename std::decay_t<Ev>::Trial tt;
    double ssq_try = 0.0;
    for (int li = 0; li < c.n_lambda; ++li) {
      double dp[4];
      ev.solve(e, c.lambdas[li], dp);
      if (norm_below(sumsq4(dp[0], dp[1], dp[2], dp[3]), c.min_step_norm)) continue;
      pt[0] = p[0] + dp[0];
      pt[1] = p[1] + dp[1];
      pt[2] = p[2] + dp[2];
      pt[3] = p[3] + dp[3];
      ssq_try = ev.trial(pt, tt);
      if (ssq_try < e.ssq) {
        found = true;
        break;
      }
    }
    if (!found) break;
    p[0] = pt[0];
    p[1] = pt[1];
    p[2] = pt[2];
    p[3] = pt[3];
    const double best_ssq = ssq_try;
    ev.accept(p, tt, e);  // coeffs(ndata, data, parm) at the accepted point (fit.py:251)
    const double change2 = sumsq4(p[0] - po0, p[1] - po1, p[2] - po2, p[3] - po3);
    if ((e.ssq - best_ssq) < c.conv_improve && norm_below(change2, c.conv_param_change)) break;
  }
  return e.ssq;
}

template <typename T>
__device__ __forceinline__ T shfl_any(T v, int src) {
  if constexpr (sizeof(T) == 8) {
    long long b = __builtin_bit_cast(long long, v);
    b = __shfl(b, src);
    return __builtin_bit_cast(T, b);
  } else {
    return __shfl(v, src);
  }
}

constexpr int kLadderLanes = 8;  // lanes per segment of the parallel-ladder descent (= the default ladder)
constexpr int kSeedShares = 8;   // FLAT 3 (the many-harmonic seed): harmonic shares per rung, 8 x 8 = the wave

// fit.py:208-258 (_run_lma_fit) with the lambda ladder evaluated in parallel. The LPS
// lanes of a lane group (lanes LPS·g .. LPS·g + LPS-1 of the wave) hold the same segment
// and the same descent state (p and coeffs at p); in every pass lane r of the group
// solves and tries rung base + r (msolve + ssqf, fit.py:226-243). The group takes the
// FIRST improving rung in ladder order, with that rung's trial state fetched from the
// lane that evaluated it, and forms coeffs there (every lane of the group, redundantly:
// same bits); if no rung of the block improved it moves to the next LPS rungs
// (n_lambda > LPS) or stops ("no lambda improved", fit.py:246-247). A rung's solve +
// trial is the same pure function of (p, J^T J, J^T r, lambda, QI) whichever lane
// computes it, and a rung whose step is below min_step_norm counts as not improving
// (the sequential ladder skips it, fit.py:230-231), so the accepted points are
// lm_descend's bit for bit; a descent costs (accepted steps + 1) passes instead of
// (accepted steps + rejected rungs + 1): at most 4 instead of 10 on config-2 segments
// (tests/test_lm_pass_structure.py). For latency-bound fits: warm-start chains
// (_fit_sequential, fitters.py:370-393) and the last segments of a record pipeline.
// Every lane of the wave must call this (wave-uniform loop; lanes without work pass
// active = false through p's group state, see lm_ladder_kernel).
// The ladder descent from a given state (p, coeffs e at p, accepted iterations `it`, the next
// rung `base` of the current iteration): lm_descend_ladder's loop. (Round 4 also resumed
// one-lane descents here that parked at their first rejected rung, lm_park_kernel: same
// bits, LM 41-45 us against 36 us, removed)
// P > 1 (the many-harmonic seed, FLAT 3): each rung is evaluated by P adjacent lanes, each over
// a share of the harmonics (PartFullEval: the P lanes of a rung end with the same bits), so the
// group is LPS x P lanes: lane = g0 + rung P + share.
template <int LPS, int P = 1, typename Ev>
__device__ __forceinline__ double lm_ladder_resume(Ev&& ev, double (&p)[4], const LMConst& c, Eval& e, int it,
                                                   int base, bool live) {
  using Trial = typename std::decay_t<Ev>::Trial;
  constexpr int NT = (int)(sizeof(Trial) / sizeof(double));
  static_assert(sizeof(Trial) == NT * sizeof(double), "trial state: doubles only");
  static_assert(LPS == 2 || LPS == 4 || LPS == 8 || LPS == 16, "LPS");
  static_assert(P == 1 || (LPS * P <= 64 && (P & (P - 1)) == 0), "P");
  const int lane = (int)__lane_id();
  const int r = (lane / P) & (LPS - 1);
  const int g0 = lane & ~(LPS * P - 1);
  bool active = live && it < c.max_steps && base < c.n_lambda;
  while (__ballot(active) != 0) {
    const int rung = base + r;
    const bool work = active && rung < c.n_lambda;
    double dp[4];
    ev.solve(e, c.lambdas[work ? rung : 0], dp);
    const bool step = work && !norm_below(sumsq4(dp[0], dp[1], dp[2], dp[3]), c.min_step_norm);
    double pt[4] = {p[0] + dp[0], p[1] + dp[1], p[2] + dp[2], p[3] + dp[3]};
    Trial tt;
    bool improved = false;
    if (step) improved = ev.trial(pt, tt) < e.ssq;
    const uint64_t imp = __ballot(improved);
    uint64_t gm;
    if constexpr (P == 1) {
      gm = (imp >> g0) & ((1ull << LPS) - 1);
    } else {  // rung k improved: its share-0 lane's bit (its P lanes agree)
      gm = 0;
#pragma unroll
      for (int k = 0; k < LPS; ++k) gm |= ((imp >> (g0 + k * P)) & 1ull) << k;
    }
    const int src = gm ? g0 + __builtin_ctzll(gm) * P + (lane & (P - 1)) : lane;
    if (__ballot(gm != 0 && active) != 0) {  // some group accepts: fetch the taken rung's state
#pragma unroll
      for (int i = 0; i < 4; ++i) pt[i] = shfl_any(pt[i], src);
      double* tv = reinterpret_cast<double*>(&tt);
#pragma unroll
      for (int i = 0; i < NT; ++i) tv[i] = shfl_any(tv[i], src);
    }
    if (active) {
      if (gm) {
        const double change2 = sumsq4(pt[0] - p[0], pt[1] - p[1], pt[2] - p[2], pt[3] - p[3]);
        p[0] = pt[0];
        p[1] = pt[1];
        p[2] = pt[2];
        p[3] = pt[3];
        const double best_ssq = ev.ssq_of(tt);  // the taken trial's ssqf
        ++it;
        base = 0;
        // as lm_descend_flat: coeffs at a point the descent stops at is needed for its ssq only
        if (((ev.ssq_of(tt) - best_ssq) < c.conv_improve && norm_below(change2, c.conv_param_change)) ||
            it >= c.max_steps) {
          e.ssq = ev.ssq_of(tt);
          active = false;
        } else {
          ev.accept(p, tt, e);  // coeffs(ndata, data, parm) at the accepted point (fit.py:251)
        }
      } else {
        base += LPS;
        if (base >= c.n_lambda) active = false;  // no lambda improved: fit.py:246-247
      }
    }
  }
  return e.ssq;
}

template <int LPS, int P = 1, typename Ev>
__device__ __forceinline__ double lm_descend_ladder(Ev&& ev, double (&p)[4], const LMConst& c, bool live = true) {
  using Trial = typename std::decay_t<Ev>::Trial;
  Eval e;
  {
    Trial t0;
    ev.trial(p, t0);
    ev.accept(p, t0, e);
  }
  return lm_ladder_resume<LPS, P>(ev, p, c, e, 0, 0, live);
}

// fit.py:260-320 (_find_best_initial_guess). jtab: n_grid rows of J_1..J_ndata(mtry)
// (psi = 0 exactly: cos(j*0) = 1, -sin(j*0) = -0). Q.qc(i) / Q.qs(i): Q_{i+1}, I_{i+1}.
// One point of fit.py:260-320's m grid (grid index g): the linear phi / amp estimates at
// mtry = M_GRID_MIN + g * step and ssqf there; false where the reference `continue`s.
template <typename QF>
DFMI_HDI bool m_grid_point(QF&& Q, int ndata, const double* __restrict__ jtab, const LMConst& c, int g,
                           double& s_out, double (&pt)[3]) {
  const double mtry = c.grid_min + (double)g * c.grid_delta;
  const double* jrow = jtab + (int64_t)g * ndata;
  double sinsum = 0.0, cossum = 0.0;
  int nsin = 0, ncos = 0;
  for (int i = 0; i < ndata; ++i) {
    const int j = i + 1;
    const double bq = jrow[i] * 1.0;   // jv * cos(j*0)
    const double bi = jrow[i] * -0.0;  // jv * -sin(j*0)
    const double dq = Q.qc(i), di = Q.qs(i);
    if (fabs(bq) > c.bessel_amp_thr) {
      switch (j & 3) {
        case 0: cossum += dq / bq; ++ncos; break;
        case 1: sinsum -= dq / bq; ++nsin; break;
        case 2: cossum -= dq / bq; ++ncos; break;
        default: sinsum += dq / bq; ++nsin; break;
      }
    }
    if (fabs(bi) > c.bessel_amp_thr) {
      switch (j & 3) {
        case 0: cossum += di / bi; ++ncos; break;
        case 1: sinsum -= di / bi; ++nsin; break;
        case 2: cossum -= di / bi; ++ncos; break;
        default: sinsum += di / bi; ++nsin; break;
      }
    }
  }
  if (nsin == 0 || ncos == 0) return false;
  const double ptry = atan2(sinsum / (double)nsin, cossum / (double)ncos);
  double sp, cp;
  sincos(ptry, &sp, &cp);
  double asum = 0.0;
  int na = 0;
  for (int i = 0; i < ndata; ++i) {
    const int j = i + 1;
    const double sc = quarter_turn(j, cp, sp);  // [cos, -sin, -cos, sin][j % 4]
    const double bq = jrow[i] * 1.0;
    const double bi = jrow[i] * -0.0;
    if (fabs(bq) > c.bessel_amp_thr && fabs(sc) > c.sincos_amp_thr) {
      asum += Q.qc(i) / (sc * bq);
      ++na;
    }
    if (fabs(bi) > c.bessel_amp_thr && fabs(sc) > c.sincos_amp_thr) {
      asum += Q.qs(i) / (sc * bi);
      ++na;
    }
  }
  if (na == 0) return false;
  const double atry = asum / (double)na;
  // ssqf at (atry, mtry, ptry, 0): fit.py:152-167 with cos(j*0)=1, sin(j*0)=0
  double s = 0.0;
  for (int i = 0; i < ndata; ++i) {
    const double common = atry * quarter_turn(i + 1, cp, sp) * jrow[i];
    const double rq = Q.qc(i) - common;
    const double ri = Q.qs(i) + common * 0.0;
    s = fma(rq, rq, s);
    s = fma(ri, ri, s);
  }
  s_out = s;
  pt[0] = atry;
  pt[1] = mtry;
  pt[2] = ptry;
  return true;
}

template <typename QF>
DFMI_HDI void m_grid_seed(QF&& Q, int ndata, const double* __restrict__ jtab, const LMConst& c, double (&best)[4]) {
  double best_ssq = 9e99;
  best[0] = best[1] = best[2] = best[3] = 0.0;
  for (int g = 0; g < c.n_grid; ++g) {
    double s, pt[3];
    if (!m_grid_point(Q, ndata, jtab, c, g, s, pt)) continue;
    if (s < best_ssq) {
      best_ssq = s;
      best[0] = pt[0];
      best[1] = pt[1];
      best[2] = pt[2];
      best[3] = 0.0;
    }
  }
}

#if defined(__HIP_DEVICE_COMPILE__)
// m_grid_seed with the grid points dealt over the L lanes of a group that runs one fit (the
// lambda-ladder descents: the seed kernels, lm_ladder_kernel): lane r evaluates points r, r + L,
// ..., keeps its first strict minimum, and the group reduces (s, g) pairs — the smaller ssq, on a
// tie the smaller grid index: exactly the serial loop's first strict minimum. Same bits, ~L
// times shorter (a seed fitted from a far guess, e.g. the quickstart's m = 31.4 from m = 6,
// always takes this path).
template <int L, typename QF>
__device__ __forceinline__ void m_grid_seed_lanes(QF&& Q, int ndata, const double* __restrict__ jtab,
                                                  const LMConst& c, double (&best)[4]) {
  const int r = (int)(__lane_id() & (L - 1));
  double bs = 9e99, bp[3] = {0.0, 0.0, 0.0};
  int bg = 0x7fffffff;
  for (int g = r; g < c.n_grid; g += L) {
    double s, pt[3];
    if (!m_grid_point(Q, ndata, jtab, c, g, s, pt)) continue;
    if (s < bs) {
      bs = s;
      bg = g;
      bp[0] = pt[0];
      bp[1] = pt[1];
      bp[2] = pt[2];
    }
  }
#pragma unroll
  for (int o = 1; o < L; o <<= 1) {
    const int src = (int)__lane_id() ^ o;
    const double os = shfl_any(bs, src);
    const int og = shfl_any(bg, src);
    const double o0 = shfl_any(bp[0], src), o1 = shfl_any(bp[1], src), o2 = shfl_any(bp[2], src);
    if (os < bs || (os == bs && og < bg)) {
      bs = os;
      bg = og;
      bp[0] = o0;
      bp[1] = o1;
      bp[2] = o2;
    }
  }
  best[0] = bp[0];
  best[1] = bp[1];
  best[2] = bp[2];
  best[3] = 0.0;
}
#endif

// fit.py:322-361 (fit): LM, status + grid retry, normalisation, phi wrap.
// Ev: the evaluator (GenSplitEval / SplitEval); FLAT = 0 runs the nested descent
// (host build / equivalence tests). Q: QI accessor for the m-grid re-seed (runtime
// harmonic index: memory, never a register array).
template <int FLAT, typename Ev>
DFMI_HDI double descend_t(Ev&& ev, double (&pp)[4], const LMConst& c) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (FLAT == 2) return lm_descend_ladder<kLadderLanes>(ev, pp, c);
  else if constexpr (FLAT == 3) return lm_descend_ladder<kLadderLanes, kSeedShares>(ev, pp, c);
  else
#endif
  if constexpr (FLAT == 1) return lm_descend_flat(ev, pp, c);
  else return lm_descend(ev, pp, c);
}

// fit.py:334-360 after the first descent (its result p, ssq): status, the m-grid re-seed
// and second descent when ssq >= FITOK_THRESHOLD, sign normalisation, phi wrap.
template <int FLAT, typename Ev, typename QF>
DFMI_HDI int fit_finish_t(Ev&& ev, QF&& Q, int ndata, const double* __restrict__ jtab, const LMConst& c,
                          double (&p)[4], double ssq, double& ssq_out) {
  auto descend = [&](double (&pp)[4]) { return descend_t<FLAT>(ev, pp, c); };
  int status;
  if (ssq < c.fitok_threshold) {
    status = 0;
  } else {
    double g[4];
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (FLAT == 2) m_grid_seed_lanes<kLadderLanes>(Q, ndata, jtab, c, g);
    else if constexpr (FLAT == 3) m_grid_seed_lanes<kLadderLanes * kSeedShares>(Q, ndata, jtab, c, g);
    else
#endif
      m_grid_seed(Q, ndata, jtab, c, g);
    if (!(g[0] == 0.0) || !(g[1] == 0.0) || !(g[2] == 0.0) || !(g[3] == 0.0)) {  // np.any
      const double ssq2 = descend(g);
      if (ssq2 < ssq) {
        ssq = ssq2;
        p[0] = g[0];
        p[1] = g[1];
        p[2] = g[2];
        p[3] = g[3];
      }
    }
    status = (ssq < c.fitok_threshold) ? 1 : 2;
  }
  const double pi = 3.141592653589793;
  if (p[0] < 0.0) {
    p[0] = -p[0];
    p[2] += pi;
  }
  if (p[1] < 0.0) {
    p[1] = -p[1];
    p[2] += pi;
  }
  p[2] = dfmi_pymod(p[2] + pi, 2.0 * pi) - pi;
  ssq_out = ssq;
  return status;
}

template <int FLAT = 1, typename Ev, typename QF>
DFMI_HDI int fit_segment_t(Ev&& ev, QF&& Q, int ndata, const double* __restrict__ jtab, const LMConst& c,
                           double (&p)[4], double& ssq_out) {
  const double ssq = descend_t<FLAT>(ev, p, c);
  return fit_finish_t<FLAT>(ev, Q, ndata, jtab, c, p, ssq, ssq_out);
}

// Single-segment entry used by the kernels and by the test-only host build.
// NDMAX > 0: register path (requires ndata <= NDMAX); NDMAX == 0: general path.
// qe: QI accessor of the LM evaluations (compile-time harmonic index after
// unrolling); qm: QI in memory for the m-grid re-seed (runtime harmonic index).
template <int NDMAX, typename QE, typename QM, int FLAT = 1>
__host__ __device__ __forceinline__ int fit_segment_q2(const QE& qe, const QM& qm, int ndata,
                                                    const double* __restrict__ jtab, const LMConst& c,
                                                    double (&p)[4], double& ssq_out) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (wide_nd(NDMAX) && FLAT == 3) {  // the many-harmonic seed: a whole wave, harmonic shares
    PartFullEval<kSeedShares, QE> ev{qe, ndata, c.trig, (int)(__lane_id() & (kSeedShares - 1))};
    return fit_segment_t<FLAT>(ev, qm, ndata, jtab, c, p, ssq_out);
  } else
#endif
  if constexpr (wide_nd(NDMAX)) {  // many harmonics: closed form over the lean Miller walk
    WideEval<QE, NDMAX == kWideNdF> ev{qe, ndata, c.trig};
    return fit_segment_t<FLAT>(ev, qm, ndata, jtab, c, p, ssq_out);
  } else if constexpr (NDMAX > 0) {
    SplitEval<NDMAX, QE> ev{qe, ndata, c.trig};
    return fit_segment_t<FLAT>(ev, qm, ndata, jtab, c, p, ssq_out);
  } else if constexpr (FLAT == 2) {  // lambda ladder: full trials (FullGenEval)
    FullGenEval<QE> ev{qe, ndata};
    return fit_segment_t<FLAT>(ev, qm, ndata, jtab, c, p, ssq_out);
  } else {  // one lane per fit: ssqf-only trials, coeffs at accepted points (GenSplitEval)
    GenSplitEval<QE> ev{qe, ndata};
    return fit_segment_t<FLAT>(ev, qm, ndata, jtab, c, p, ssq_out);
  }
}

template <int NDMAX, typename QF, int FLAT = 1>
__host__ __device__ __forceinline__ int fit_segment_q(const QF& q, int ndata, const double* __restrict__ jtab,
                                                   const LMConst& c, double (&p)[4], double& ssq_out) {
  return fit_segment_q2<NDMAX, QF, QF, FLAT>(q, q, ndata, jtab, c, p, ssq_out);
}

// Component-major QI (qi[c·ld + s], qptr = qi + s). QI is re-read per evaluation
// through the vector L1 (64 segments x 2·ndata doubles = 10 KB per wave): keeping
// it in registers costs 2·NDMAX VGPRs and with them the second wave per SIMD.
template <int NDMAX, int FLAT = 1, int PRE = 0>
__host__ __device__ __forceinline__ int fit_segment(const double* __restrict__ qptr, int64_t ld, int ndata,
                                                 const double* __restrict__ jtab, const LMConst& c, double (&p)[4],
                                                 double& ssq_out) {
  const QGlobalT<PRE> qg{qptr, ld, ndata};
  return fit_segment_q<NDMAX, QGlobalT<PRE>, FLAT>(qg, ndata, jtab, c, p, ssq_out);
}

// Seeds of up to 8 records passed by value (read with constant offsets only).
struct GuessInline {
  double v[8][4];
};

// One lane per chunk. Records r < nrec each hold nbuf segments; the fitted
// items of record r are segments [first, first + nitems); they are cut into
// nchunk chunks with np.array_split semantics and each chunk starts from the
// record's guess, warm-starting within the chunk (fitters.py:42-58).
// Guess source: ginl (use_inline) or guess[r*g_rec + i*g_comp].
// CHAIN = false: every chunk holds at most one segment (no loop: the register
// allocator keeps the whole LM at two waves per SIMD); CHAIN = true: warm-start
// chains of any length.
// ROWS = false: QI component-major (qi[c·qi_ld + s]); the demodulation wrote dc.
// ROWS = true (CHAIN = false only): QI as demodulation rows (qi + s·qi_ld, see
// dfmi_qi_row_stride); the kernel also copies each segment's dc into out[4].
// With the register path the wave first stages its 64 rows into LDS, transposed
// ([pos][65]: conflict-free column reads), with coalesced 16-B loads when the
// rows are contiguous — each QI value is then read from LDS at every evaluation.
// QREG (exact-ndata register path, chunk size 1): the segment's QI values are loaded
// into registers once (QRegs) instead of re-read from LDS / L1 at every evaluation
// (ndata 10: 248 VGPRs, still 2 waves per SIMD; step 0.5558 -> 0.5507 ms,
// profiles/r02m_tune_lm_spec3.log). Same bits either way.
// Waves per SIMD the chunk-size-1 12-harmonic variant is compiled for: 2 (280 -> 256 VGPRs, 29
// spilled) runs dfmi_lm at ndata 12 in 0.047 ms per 100k segments against 0.055 at one wave;
// the 16-harmonic variant spills ~240 values at 2 and runs 2.5x slower (0.171 vs 0.068 ms,
// r05as), so it keeps its allocation.
template <int NDMAX, bool CHAIN, bool ONEPASS = false>
constexpr int lm_waves() {
  return (!CHAIN && (NDMAX == 12 || ONEPASS || wide_nd(NDMAX))) ? 2 : 1;  // ONEPASS: 259 VGPRs unbounded
}
// ONEPASS (general path, chunk size 1, component-major): each lane keeps its Bessel recurrence
// values in dynamic LDS (64 x (ndata + 2) doubles per wave) and walks once per evaluation
// (harmonic_walk_q); same bits.
template <int NDMAX, bool CHAIN, bool ROWS = false, bool QREG = false, bool ONEPASS = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(lm_waves<NDMAX, CHAIN, ONEPASS>()))) void lm_chunks_kernel(
    const double* __restrict__ qi, int64_t qi_ld, int ndata, int64_t nrec, int64_t nbuf, int64_t first,
    int64_t nitems, int64_t nchunk, const double* __restrict__ guess, int64_t g_rec, int64_t g_comp,
    GuessInline ginl, int use_inline, const double* __restrict__ jtab, LMConst c, double* __restrict__ out,
    int64_t out_ld, int32_t* __restrict__ status) {
  static_assert(!(ROWS && CHAIN), "row layout: chunk size 1 only");
  constexpr bool kQReg = QREG && nd_exact(NDMAX) && !CHAIN;
  extern __shared__ double lds_q[];  // STAGE: [qi_ld][65]
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool valid = id < nrec * nchunk;
  const int64_t idc = valid ? id : 0;
  const int64_t r = idc / nchunk;
  const int64_t k = idc - r * nchunk;
  const int64_t qn = nitems / nchunk, rm = nitems % nchunk;
  const int64_t start = k * qn + (k < rm ? k : rm);
  const int64_t len = qn + (k < rm ? 1 : 0);
  const int64_t s0 = r * nbuf + first + start;
  constexpr bool STAGE = ROWS && NDMAX > 0;
  if constexpr (STAGE) {
    const int lane = threadIdx.x;
    const int QS = (int)qi_ld;
    const int64_t sl0 = __shfl(s0, 0);  // lane 0 is always valid
    const int nv = (int)((nrec * nchunk - (int64_t)blockIdx.x * 64) < 64 ? (nrec * nchunk - (int64_t)blockIdx.x * 64)
                                                                         : 64);
    const bool contiguous = __all(!valid || s0 == sl0 + lane);
    if (contiguous) {
      const double* __restrict__ base = qi + sl0 * qi_ld;
      const int tot = nv * QS;  // doubles, even
      // groups of kStageLoads 16-B loads issued together, then written to LDS: one memory
      // round trip per 16 KB (64 rows of 32 doubles) instead of one per 1-KB load
      constexpr int kStageLoads = 16;
      typedef double d2v __attribute__((ext_vector_type(2)));
      for (int e0 = 2 * lane; e0 < tot; e0 += 128 * kStageLoads) {
        d2v v[kStageLoads];
#pragma unroll
        for (int u = 0; u < kStageLoads; ++u) {
          const int e = e0 + 128 * u;
          v[u] = e < tot ? *reinterpret_cast<const d2v*>(base + e) : d2v{0.0, 0.0};
        }
#pragma unroll
        for (int u = 0; u < kStageLoads; ++u) {
          const int e = e0 + 128 * u;
          if (e < tot) {
            const int row = e / QS, pos = e - row * QS;
            lds_q[pos * 65 + row] = v[u].x;
            lds_q[(pos + 1) * 65 + row] = v[u].y;
          }
        }
      }
    } else if (valid) {
      for (int pos = 0; pos < QS; ++pos) lds_q[pos * 65 + lane] = qi[s0 * qi_ld + pos];
    }
    __syncthreads();
  }
  if (!valid) return;
  double p[4] = {0.0, 0.0, 0.0, 0.0};
  if (use_inline) {
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
      if (r == rr) {
#pragma unroll
        for (int i = 0; i < 4; ++i) p[i] = ginl.v[rr][i];
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = guess[r * g_rec + i * g_comp];
  }
  auto put = [&](int64_t sidx, int st, double ssq) {
    out[0 * out_ld + sidx] = p[0];
    out[1 * out_ld + sidx] = p[1];
    out[2 * out_ld + sidx] = p[2];
    out[3 * out_ld + sidx] = p[3];
    out[5 * out_ld + sidx] = ssq;
    status[sidx] = st;
  };
  if constexpr (ROWS) {
    if (len != 1) return;
    double ssq;
    int st;
    double dcv;
    if constexpr (STAGE) {
      const QRow<65> q{lds_q + threadIdx.x};  // QI read from LDS at every evaluation
      if constexpr (kQReg) {
        QRegs<nd_cap(NDMAX)> qr;
        qr.load(q);
        st = fit_segment_q2<NDMAX, QRegs<nd_cap(NDMAX)>, QRow<65>, 1>(qr, q, ndata, jtab, c, p, ssq);
      } else {
        st = fit_segment_q<NDMAX, QRow<65>>(q, ndata, jtab, c, p, ssq);
      }
      dcv = q.at(dfmi_row_dc(ndata));
    } else {
      const QRow<1> q{qi + s0 * qi_ld};
      st = fit_segment_q<NDMAX>(q, ndata, jtab, c, p, ssq);
      dcv = q.at(dfmi_row_dc(ndata));
    }
    put(s0, st, ssq);
    out[4 * out_ld + s0] = dcv;
    // first == 1: the record's seed buffer was fitted elsewhere (the fused seed kernel): carry
    // its dc. (A launch over a later slice of the buffers, first > 1, leaves the segments
    // before it to the launch that fitted them: nls_record_hostout's tail.)
    if (k == 0 && first == 1) out[4 * out_ld + r * nbuf] = qi[r * nbuf * qi_ld + dfmi_row_dc(ndata)];
  } else {
    auto one = [&](int64_t sidx) {
      double ssq;
      int st;
      if constexpr (wide_nd(NDMAX) && QREG && !CHAIN) {
        // the lane's 2 ndata QI into its own LDS column (no other lane reads it: no barrier),
        // 16 loads in flight
        double* col = lds_q + threadIdx.x;
        const double* __restrict__ src = qi + sidx;
        const int nc = 2 * ndata;
        for (int c0 = 0; c0 < nc; c0 += 16) {
          double v[16];
#pragma unroll
          for (int u = 0; u < 16; ++u) v[u] = c0 + u < nc ? src[(int64_t)(c0 + u) * qi_ld] : 0.0;
#pragma unroll
          for (int u = 0; u < 16; ++u)
            if (c0 + u < nc) col[(c0 + u) * 64] = v[u];
        }
        const QLds ql{col, ndata};
        st = fit_segment_q<NDMAX, QLds, 1>(ql, ndata, jtab, c, p, ssq);
      } else if constexpr (wide_nd(NDMAX)) {
        const QCol qg{qi, (uint32_t)sidx, qi_ld, ndata};
        st = fit_segment_q<NDMAX, QCol, 1>(qg, ndata, jtab, c, p, ssq);
      } else if constexpr (kQReg) {
        const QGlobal qg{qi + sidx, qi_ld, ndata};
        QRegs<nd_cap(NDMAX)> qr;
        qr.load(qg);
        st = fit_segment_q2<NDMAX, QRegs<nd_cap(NDMAX)>, QGlobal, 1>(qr, qg, ndata, jtab, c, p, ssq);
      } else if constexpr (ONEPASS && NDMAX == 0 && !CHAIN && !ROWS) {
        const QGlobalT<kQPre, true> qg{qi + sidx, qi_ld, ndata, lds_q + threadIdx.x};
        st = fit_segment_q<NDMAX, QGlobalT<kQPre, true>, 1>(qg, ndata, jtab, c, p, ssq);
      } else {
        st = fit_segment<NDMAX, 1, CHAIN ? 0 : kQPre>(qi + sidx, qi_ld, ndata, jtab, c, p, ssq);
      }
      put(sidx, st, ssq);
    };
    if constexpr (!CHAIN) {
      if (len == 1) one(s0);  // chunk size 1 (the parallel default): straight-line code
    } else {
      for (int64_t t = 0; t < len; ++t) one(s0 + t);  // warm-start chain (sequential / n_cores)
    }
  }
}

// Many harmonics with P lanes per segment (PartEval): chunk size 1 (every segment its own
// chunk, seeded by its record's guess), component-major QI staged into a per-wave LDS tile
// [2 ndata][64 / P] (dynamic LDS), lane r = threadIdx.x % P of each group writing nothing but
// its share of the sums, lane 0 the results. Items and guesses as lm_chunks_kernel.
template <int P>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void lm_split_kernel(
    const double* __restrict__ qi, int64_t qi_ld, int ndata, int64_t nrec, int64_t nbuf, int64_t first,
    int64_t nitems, const double* __restrict__ guess, int64_t g_rec, int64_t g_comp, GuessInline ginl, int use_inline,
    const double* __restrict__ jtab, LMConst c, double* __restrict__ out, int64_t out_ld, int32_t* __restrict__ status) {
  extern __shared__ double lds_q[];
  constexpr int G = 64 / P;  // segments per wave
  const int lane = threadIdx.x, gi = lane / P, r = lane % P;
  const int64_t id = (int64_t)blockIdx.x * G + gi;
  const bool valid = id < nrec * nitems;
  const int64_t idc = valid ? id : 0;
  const int64_t rec = idc / nitems;
  const int64_t sidx = rec * nbuf + first + (idc - rec * nitems);
  double* col = lds_q + gi;
  const int nc = 2 * ndata;
  if (valid) {  // the group's P lanes load the segment's components r, r + P, ... (8 in flight)
    const double* __restrict__ src = qi + sidx;
    for (int c0 = r; c0 < nc; c0 += 8 * P) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = c0 + u * P < nc ? src[(int64_t)(c0 + u * P) * qi_ld] : 0.0;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (c0 + u * P < nc) col[(c0 + u * P) * G] = v[u];
    }
  }
  __syncthreads();  // one wave: the tile is read by every lane of a group
  if (!valid) return;  // a group is valid or not as a whole
  double p[4] = {0.0, 0.0, 0.0, 0.0};
  if (use_inline) {
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
      if (rec == rr) {
#pragma unroll
        for (int i = 0; i < 4; ++i) p[i] = ginl.v[rr][i];
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = guess[rec * g_rec + i * g_comp];
  }
  const QLdsG<G> q{col, ndata};
  PartEval<P, QLdsG<G>> ev{q, ndata, c.trig, r};
  double ssq;
  const int st = fit_segment_t<1>(ev, q, ndata, jtab, c, p, ssq);
  if (r != 0) return;
  out[0 * out_ld + sidx] = p[0];
  out[1 * out_ld + sidx] = p[1];
  out[2 * out_ld + sidx] = p[2];
  out[3 * out_ld + sidx] = p[3];
  out[5 * out_ld + sidx] = ssq;
  status[sidx] = st;
}

// Latency-bound fits (few chains or few segments): kLadderLanes lanes per item, the
// lambda ladder of every LM iteration tried in one pass (lm_descend_ladder). Items and
// chunks as lm_chunks_kernel (np.array_split chunks of the record's segments
// [first, first + nitems), warm start within a chunk, fitters.py:13-60); ROWS: QI as
// demodulation rows (chunk size 1; dc copied into out[4] as lm_chunks_kernel does).
// Lane 0 of each group writes the results. A wave holds 64 / kLadderLanes items.
// LPSI = 64 (many harmonics, the one-walk evaluator: tuning lm_ladder_split): one item per wave,
// each λ rung evaluated by 8 lanes over harmonic shares (FLAT 3, as the seed), the segment's QI
// staged in LDS for every fit.
template <int NDMAX, bool CHAIN, bool ROWS, int LPSI = kLadderLanes>
__global__ __launch_bounds__(64) void lm_ladder_kernel(
    const double* __restrict__ qi, int64_t qi_ld, int ndata, int64_t nrec, int64_t nbuf, int64_t first,
    int64_t nitems, int64_t nchunk, const double* __restrict__ guess, int64_t g_rec, int64_t g_comp,
    GuessInline ginl, int use_inline, const double* __restrict__ jtab, LMConst c, double* __restrict__ out,
    int64_t out_ld, int32_t* __restrict__ status) {
  static_assert(!(ROWS && CHAIN), "row layout: chunk size 1 only");
  static_assert(LPSI == kLadderLanes || (LPSI == 64 && wide_nd(NDMAX) && !ROWS), "wave-split ladder");
  constexpr int LPS = LPSI;
  constexpr int FL = LPSI == 64 ? 3 : 2;
  constexpr bool kQReg = NDMAX > 0 && nd_exact(NDMAX);
  const int64_t id = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / LPS;
  if (id >= nrec * nchunk) return;  // whole groups leave together
  const bool lead = (threadIdx.x & (LPS - 1)) == 0;
  const int64_t r = id / nchunk;
  const int64_t k = id - r * nchunk;
  const int64_t qn = nitems / nchunk, rm = nitems % nchunk;
  const int64_t start = k * qn + (k < rm ? k : rm);
  const int64_t len = qn + (k < rm ? 1 : 0);
  const int64_t s0 = r * nbuf + first + start;
  double p[4] = {0.0, 0.0, 0.0, 0.0};
  if (use_inline) {
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) {
      if (r == rr) {
#pragma unroll
        for (int i = 0; i < 4; ++i) p[i] = ginl.v[rr][i];
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = guess[r * g_rec + i * g_comp];
  }
  auto fit = [&](const auto& qm, int64_t sidx) {
    double ssq;
    int st;
    if constexpr (kQReg) {
      QRegs<nd_cap(NDMAX)> qr;
      qr.load(qm);
      st = fit_segment_q2<NDMAX, QRegs<nd_cap(NDMAX)>, std::decay_t<decltype(qm)>, 2>(qr, qm, ndata, jtab, c, p, ssq);
    } else {
      st = fit_segment_q2<NDMAX, std::decay_t<decltype(qm)>, std::decay_t<decltype(qm)>, FL>(qm, qm, ndata, jtab, c, p,
                                                                                           ssq);
    }
    if (lead) {
      out[0 * out_ld + sidx] = p[0];
      out[1 * out_ld + sidx] = p[1];
      out[2 * out_ld + sidx] = p[2];
      out[3 * out_ld + sidx] = p[3];
      out[5 * out_ld + sidx] = ssq;
      status[sidx] = st;
    }
  };
  if constexpr (ROWS) {
    if (len != 1) return;
    const QRow<1> q{qi + s0 * qi_ld};
    fit(q, s0);
    if (lead) {
      out[4 * out_ld + s0] = q.at(dfmi_row_dc(ndata));
      if (k == 0 && first == 1)  // the seed buffer was fitted elsewhere: carry its dc (lm_chunks_kernel)
        out[4 * out_ld + r * nbuf] = qi[r * nbuf * qi_ld + dfmi_row_dc(ndata)];
    }
  } else if constexpr (kQReg && CHAIN) {
    // warm-start chain (sequential / n_cores). Every LPS fits the group stages the QI of
    // its next LPS segments into LDS, one segment per lane with all 2·ndata loads in
    // flight: one memory latency per LPS fits instead of one per fit (the fits themselves
    // read no global memory). The m-grid re-seed keeps its global accessor.
    constexpr int NC = nd_cap(NDMAX);
    __shared__ double stage[64 / LPS][LPS][2 * NC];
    const int g = (int)(threadIdx.x / LPS), gl = (int)(threadIdx.x & (LPS - 1));
    for (int64_t t = 0; t < len; ++t) {
      const int slot = (int)(t & (LPS - 1));
      if (slot == 0) {
        if (t + gl < len) {
          const double* __restrict__ qs = qi + s0 + t + gl;
          double v[2 * NC];
#pragma unroll
          for (int cc = 0; cc < 2 * NC; ++cc) v[cc] = qs[(int64_t)cc * qi_ld];
#pragma unroll
          for (int cc = 0; cc < 2 * NC; ++cc) stage[g][gl][cc] = v[cc];
        }
        // one wave: its LDS operations run in order; the fence keeps the compiler from
        // moving the reads below above the other lanes' writes
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      QRegs<NC> qr;
#pragma unroll
      for (int h = 0; h < NC; ++h) {
        qr.c[h] = stage[g][slot][h];
        qr.s[h] = stage[g][slot][NC + h];
      }
      const QGlobal q{qi + s0 + t, qi_ld, ndata};
      double ssq;
      const int st = fit_segment_q2<NDMAX, QRegs<NC>, QGlobal, 2>(qr, q, ndata, jtab, c, p, ssq);
      if (lead) {
        out[0 * out_ld + s0 + t] = p[0];
        out[1 * out_ld + s0 + t] = p[1];
        out[2 * out_ld + s0 + t] = p[2];
        out[3 * out_ld + s0 + t] = p[3];
        out[5 * out_ld + s0 + t] = ssq;
        status[s0 + t] = st;
      }
    }
  } else if constexpr (LPSI == 64) {
    // one segment per wave: its QI into LDS (2 ndata doubles; beyond 128 harmonics from global)
    __shared__ double qsh[2 * 128];
    for (int64_t t = 0; t < len; ++t) {
      if (ndata <= 128) {
        __builtin_amdgcn_wave_barrier();  // the previous fit's reads are done (one wave, in order)
        for (int i = (int)threadIdx.x; i < 2 * ndata; i += 64) qsh[i] = qi[(int64_t)i * qi_ld + s0 + t];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      const QGlobal q{ndata <= 128 ? qsh : qi + s0 + t, ndata <= 128 ? 1 : qi_ld, ndata};
      fit(q, s0 + t);
    }
  } else {
    for (int64_t t = 0; t < len; ++t) {  // warm-start chain (sequential / n_cores); len 1: chunk size 1
      const QGlobal q{qi + s0 + t, qi_ld, ndata};
      fit(q, s0 + t);
    }
  }
}

}  // namespace dfmi
