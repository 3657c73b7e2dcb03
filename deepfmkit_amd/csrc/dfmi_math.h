// dfmi_math.h — fp64 math shared by the HIP kernels and the host side of libdfmi.
//
// Integer-order Bessel functions J_k(x), k = 0..N, by Miller's backward
// recurrence, evaluated in TWO identical passes so that no per-lane array is
// needed on the GPU:
//   pass 1 (bessel_norm) runs the recurrence from the start order down to 0 and
//          returns the normalisation S = f_0 + 2 sum f_2k (Neumann identity);
//   pass 2 (BesselWalk)  re-runs the SAME recurrence (same rounding, same
//          rescale events) and hands out J_{k+1}, J_k, J_{k-1} at each order
//          k = N..1, already normalised.
// Overflow: whenever |f| exceeds 2^600 all live values (and S in pass 1) are
// multiplied by 2^-600 — an exact power-of-two scaling — and an exponent
// counter is bumped; values from an earlier scale are mapped to the final
// scale with ldexp, which is again exact (or underflows to 0, which is the
// right answer for those orders).
//
// This replaces scipy.special.jv, the third-party Bessel the reference calls at
// fit.py:106,108,160,275-276. Accuracy against the
// scipy 1.15.3 table in tests/golden/bessel.npz: tests/test_host_numerics.py::test_bessel_vs_scipy_table
// (host build) and tests/test_gpu_numerics.py (device).
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define DFMI_HD __host__ __device__ __forceinline__
#else
#define DFMI_HD static inline
#endif

#define DFMI_BES_BIG_EXP 600

// Demodulation row layout of the record pipeline (demod.h fold_finish ROWS, lm.h
// QRow): one row of dfmi_qi_row_stride(ndata) doubles per segment; per block of
// 8 harmonics 16 doubles [Q_{8b+1..8b+8} | I_{8b+1..8b+8}] — exactly one 128-B
// line, written by one store instruction — and dc = mean(segment) in the first
// unused Q slot of the last block (an extra 8-double tail when ndata % 8 == 0).
DFMI_HD int dfmi_row_stride(int ndata) {
  const int nblk = (ndata + 7) / 8;
  return 16 * nblk + ((ndata % 8) ? 0 : 8);
}
DFMI_HD int dfmi_row_dc(int ndata) {
  const int nblk = (ndata + 7) / 8;
  return (ndata % 8) ? 16 * (nblk - 1) + (ndata % 8) : 16 * nblk;
}

// Start order of the backward recurrence (even). Fitted to the minimal order at
// which the truncation error sinks below the fp64 rounding floor (checked against
// mpmath for N <= 63, |x| <= 64): M = max(N + 10, 1.1|x| + 14 + 3 sqrt|x|).
DFMI_HD int dfmi_bessel_start(int N, double ax) {
  const double mx = 1.1 * ax + 14.0 + 3.0 * sqrt(ax);
  int M = (int)mx + 1;
  if (M < N + 10) M = N + 10;
  return (M + 1) & ~1;
}

// Pass 1: normalisation S at the final scale, and the final scale exponent.
DFMI_HD double dfmi_bessel_norm(double ax, int M, int* e_final) {
  const double two_over_x = 2.0 / ax;
  const double big = ldexp(1.0, DFMI_BES_BIG_EXP);
  double fp1 = 0.0, f = 1.0, S = 0.0;
  int e = 0;
  // order M is even: it contributes 2*f_M
  S = 2.0 * f;
  for (int k = M; k >= 1; --k) {
    double fm1 = fma((double)k * two_over_x, f, -fp1);  // f_{k-1}
    if (fabs(fm1) > big) {
      fm1 = ldexp(fm1, -DFMI_BES_BIG_EXP);
      f = ldexp(f, -DFMI_BES_BIG_EXP);
      S = ldexp(S, -DFMI_BES_BIG_EXP);
      ++e;
    }
    const int km1 = k - 1;
    if (km1 == 0) S += fm1;
    else if ((km1 & 1) == 0) S += 2.0 * fm1;
    fp1 = f;
    f = fm1;
  }
  *e_final = e;
  return S;
}

// Pass 1 that also keeps the raw values f_0..f_nmax (store[k * stride], as formed): when no
// rescale happened (*e_final == 0) they are exactly the values pass 2 would form again, so
// J_k = f_k * (1 / S) can be read back instead of walking a second time (lm.h
// harmonic_walk_q); with a rescale the caller walks as usual.
DFMI_HD double dfmi_bessel_norm_store(double ax, int M, int* e_final, double* store, int stride, int nmax) {
  const double two_over_x = 2.0 / ax;
  const double big = ldexp(1.0, DFMI_BES_BIG_EXP);
  double fp1 = 0.0, f = 1.0, S = 0.0;
  int e = 0;
  S = 2.0 * f;
  for (int k = M; k >= 1; --k) {
    double fm1 = fma((double)k * two_over_x, f, -fp1);  // f_{k-1}
    if (fabs(fm1) > big) {
      fm1 = ldexp(fm1, -DFMI_BES_BIG_EXP);
      f = ldexp(f, -DFMI_BES_BIG_EXP);
      S = ldexp(S, -DFMI_BES_BIG_EXP);
      ++e;
    }
    const int km1 = k - 1;
    if (km1 == nmax) store[(k) * stride] = f;  // f_{nmax + 1}
    if (km1 <= nmax) store[km1 * stride] = fm1;
    if (km1 == 0) S += fm1;
    else if ((km1 & 1) == 0) S += 2.0 * fm1;
    fp1 = f;
    f = fm1;
  }
  *e_final = e;
  return S;
}

// Pass 2: walk k = M..1; at each k the caller gets J_{k+1}, J_k, J_{k-1}.
struct DfmiBesselWalk {
  double two_over_x, big, invS, fp1, f;
  int e, e_final, k;
  bool neg;
  DFMI_HD void init(double x, int M, double S, int e_fin) {
    neg = x < 0.0;
    const double ax = fabs(x);
    two_over_x = 2.0 / ax;
    big = ldexp(1.0, DFMI_BES_BIG_EXP);
    invS = 1.0 / S;
    fp1 = 0.0;
    f = 1.0;
    e = 0;
    e_final = e_fin;
    k = M;
  }
  // Advance one order: afterwards (jp1, j0, jm1) = J_{k+1}, J_k, J_{k-1} for the
  // order k the walk was at BEFORE the call (then k is decremented).
  DFMI_HD int step(double* jp1, double* j0, double* jm1) {
    double fm1 = fma((double)k * two_over_x, f, -fp1);  // identical to pass 1
    double a = fp1, b = f;
    if (fabs(fm1) > big) {
      fm1 = ldexp(fm1, -DFMI_BES_BIG_EXP);
      a = ldexp(a, -DFMI_BES_BIG_EXP);
      b = ldexp(b, -DFMI_BES_BIG_EXP);
      f = b;
      ++e;
    }
    const int sh = -DFMI_BES_BIG_EXP * (e_final - e);
    double vp1 = a * invS, v0 = b * invS, vm1 = fm1 * invS;
    if (sh != 0) {
      vp1 = ldexp(vp1, sh);
      v0 = ldexp(v0, sh);
      vm1 = ldexp(vm1, sh);
    }
    const int kk = k;
    if (neg) {  // J_n(-x) = (-1)^n J_n(x)
      if ((kk + 1) & 1) vp1 = -vp1;
      if (kk & 1) v0 = -v0;
      if ((kk - 1) & 1) vm1 = -vm1;
    }
    *jp1 = vp1;
    *j0 = v0;
    *jm1 = vm1;
    fp1 = f;
    f = fm1;
    --k;
    return kk;
  }
};

// Tiny argument (|x| < 1e-8): two terms of the power series,
// J_k(x) = (x/2)^k / k! * (1 - (x/2)^2/(k+1)), relative error < 1e-33. The
// backward recurrence would overflow there (one step grows by 2k/|x|).
#define DFMI_BES_TINY 1e-8
DFMI_HD double dfmi_bessel_series(int k, double x) {
  const double h = 0.5 * x;
  double t = 1.0;
  for (int i = 1; i <= k; ++i) t *= h / (double)i;
  return t * (1.0 - h * h / (double)(k + 1));
}

// Large arguments: the backward recurrence starts ~1.1|x| orders up, so at |x| ~ 900 (a
// descent running away from a guess that cannot reach the data, the seed of DESIGN.md §4)
// one evaluation walks ~1,000 orders twice. For |x| >= DFMI_BES_LARGE with the wanted orders
// below |x| / 2: J_0, J_1 by their Hankel asymptotic expansions (Abramowitz & Stegun
// 9.2.5-9.2.10: J_n = sqrt(2 / (pi x)) (P cos chi - Q sin chi), chi = x - (n/2 + 1/4) pi,
// P, Q series in 1/x with a_k = prod_{i<=k} (4n^2 - (2i-1)^2) / (k! 8^k), 7 terms each: the
// next term is < 1e-17 relative at |x| = 64), then J_{k+1} = (2k / x) J_k - J_{k-1} upward
// (no dominant solution for k < |x|: errors grow ~ k eps). Measured against mpmath for
// |x| in [64, 5000], orders 0..13: max abs error 4.2e-17 (scripts/study notes,
// tests/test_host_numerics.py::test_bessel_large_argument_vs_scipy). The phase uses
// sincos(x) (Cody-Waite in three parts: exact reduction for |x| < 2^19) rotated by pi/4, not
// sincos(x - pi/4), whose argument would carry x's rounding.
#define DFMI_BES_LARGE 64.0
DFMI_HD void dfmi_sincos_fast(double x, double* sn, double* cs);
DFMI_HD bool dfmi_bessel_use_large(double ax, int N) { return ax >= DFMI_BES_LARGE && 2.0 * (double)(N + 1) <= ax; }

DFMI_HD void dfmi_bessel_j01_large(double ax, double* j0, double* j1) {
  const double z = 1.0 / ax, z2 = z * z;
  // (-1)^k a_{2k}(n) and (-1)^k a_{2k+1}(n), n = 0, 1 (exact rationals rounded once)
  const double p0 = fma(z2, fma(z2, fma(z2, fma(z2, fma(z2, fma(z2, 3038.090510922384, -110.01714026924674),
                                                       6.074042001273483), -0.5725014209747314),
                                      0.112152099609375), -0.0703125), 1.0);
  const double q0 = z * fma(z2, fma(z2, fma(z2, fma(z2, fma(z2, fma(z2, -18257.755474293175, 551.3358961220206),
                                                            -24.380529699556064), 1.7277275025844574),
                                           -0.22710800170898438), 0.0732421875), -0.125);
  const double p1 = fma(z2, fma(z2, fma(z2, fma(z2, fma(z2, fma(z2, -3302.2722944808525, 121.59789187653587),
                                                       -6.883914268109947), 0.6765925884246826),
                                      -0.144195556640625), 0.1171875), 1.0);
  const double q1 = z * fma(z2, fma(z2, fma(z2, fma(z2, fma(z2, fma(z2, 19718.37591223663, -603.8440767050702),
                                                            27.248827311268542), -1.993531733751297),
                                           0.2775764465332031), -0.1025390625), 0.375);
  double sn, cs;
  dfmi_sincos_fast(ax, &sn, &cs);  // ax < 1e5 (callers): the exact three-part reduction
  const double r = 0.70710678118654752440;
  const double c0 = (cs + sn) * r, s0 = (sn - cs) * r;  // cos, sin (x - pi/4)
  const double c1 = (sn - cs) * r, s1 = -(sn + cs) * r; // cos, sin (x - 3 pi/4)
  const double amp = sqrt(0.63661977236758134308 * z);  // sqrt(2 / (pi x))
  *j0 = amp * fma(p0, c0, -(q0 * s0));
  *j1 = amp * fma(p1, c1, -(q1 * s1));
}

// Convenience (host tests / tables): J_0..J_N(x) into out[0..N].
DFMI_HD void dfmi_bessel_table(double x, int N, double* out) {
  if (x == 0.0) {
    out[0] = 1.0;
    for (int k = 1; k <= N; ++k) out[k] = 0.0;
    return;
  }
  const double ax = fabs(x);
  if (!(ax < 1.0e5)) {  // NaN or absurd argument
    for (int k = 0; k <= N; ++k) out[k] = __builtin_nan("");
    return;
  }
  if (ax < DFMI_BES_TINY) {
    for (int k = 0; k <= N; ++k) out[k] = dfmi_bessel_series(k, x);
    return;
  }
  if (dfmi_bessel_use_large(ax, N)) {
    double jm1, j0;
    dfmi_bessel_j01_large(ax, &jm1, &j0);
    const double tox = 2.0 / ax;
    out[0] = jm1;
    if (N >= 1) out[1] = x < 0.0 ? -j0 : j0;
    for (int k = 1; k < N; ++k) {
      const double jp1 = fma((double)k * tox, j0, -jm1);
      out[k + 1] = (x < 0.0 && ((k + 1) & 1)) ? -jp1 : jp1;
      jm1 = j0;
      j0 = jp1;
    }
    return;
  }
  const int M = dfmi_bessel_start(N, ax);
  int ef = 0;
  const double S = dfmi_bessel_norm(ax, M, &ef);
  DfmiBesselWalk w;
  w.init(x, M, S, ef);
  for (int k = M; k >= 1; --k) {
    double jp1, j0, jm1;
    w.step(&jp1, &j0, &jm1);
    if (k - 1 <= N) out[k - 1] = jm1;
    if (k <= N) out[k] = j0;
  }
}

// fmod(a, b) for b > 0 and |a| < 2^40 b, exactly (fmod's result is always representable,
// so one fma with the right integer quotient k gives it with no rounding): k from
// a * (1/b), whose relative error cannot move trunc by more than one, then corrected by
// the sign / range of the remainder. The library fmod is an iterative (bitwise) loop on
// the device.
DFMI_HD double dfmi_fmod_pos(double a, double b) {
  double k = trunc(a * (1.0 / b));
  double r = fma(-k, b, a);
  if (a >= 0.0) {
    if (r < 0.0) k -= 1.0;
    else if (r >= b) k += 1.0;
  } else {
    if (r > 0.0) k += 1.0;
    else if (r <= -b) k -= 1.0;
  }
  r = fma(-k, b, a);
  return r == 0.0 ? copysign(0.0, a) : r;
}

// numpy float64 modulo (npy_divmod): result has the sign of the divisor.
DFMI_HD double dfmi_pymod(double a, double b) {
  double mod = (b > 0.0 && fabs(a) < 1.0995116277760000e12 * b) ? dfmi_fmod_pos(a, b) : fmod(a, b);
  if (mod != 0.0) {
    if ((b < 0.0) != (mod < 0.0)) mod += b;
  } else {
    mod = copysign(0.0, b);
  }
  return mod;
}

// sin/cos for |x| < 2^19 without branches: Cody-Waite reduction by pi/2 in three
// parts, fdlibm kernel polynomials on [-pi/4, pi/4], quadrant by select. Callers
// use the library sincos for larger arguments (|x| >= 2^19; dfmi_sincos below).
DFMI_HD void dfmi_sincos_fast(double x, double* sn, double* cs) {
  const double invpio2 = 6.36619772367581382433e-01;
  const double p1 = 1.57079632673412561417e+00, p2 = 6.07710050630396597660e-11, p3 = 2.02226624871116645580e-21;
  const double q = rint(x * invpio2);
  double r = fma(-q, p1, x);
  r = fma(-q, p2, r);
  r = fma(-q, p3, r);
  const double z = r * r;
  const double ps = fma(z, fma(z, fma(z, fma(z, fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                                              2.75573137070700676789e-06), -1.98412698298579493134e-04),
                             8.33333333332248946124e-03), -1.66666666666666324348e-01);
  const double sr = fma(r * z, ps, r);
  const double pc = fma(z, fma(z, fma(z, fma(z, fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                              -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                             -1.38888888888741095749e-03), 4.16666666666666019037e-02);
  const double cr = fma(z * z, pc, fma(-0.5, z, 1.0));
  const int qi = ((int)q) & 3;
  *sn = (qi == 0) ? sr : (qi == 1) ? cr : (qi == 2) ? -sr : -cr;
  *cs = (qi == 0) ? cr : (qi == 1) ? -sr : (qi == 2) ? -cr : sr;
}

#if defined(__HIP_DEVICE_COMPILE__)
// The library's large-argument sincos (Payne-Hanek: table loads from global memory)
// kept out of line: inlined, its loads make the compiler wait for every vector memory
// operation in flight (prefetched samples included) where its branch rejoins the fast
// path, on every call, taken or not.
static __device__ __noinline__ double2 dfmi_sincos_lib(double x) {
  double s, c;
  sincos(x, &s, &c);
  return make_double2(s, c);
}
#endif

// dfmi_sincos_fast's constants as a runtime value (a kernel argument: uniform, so they
// live in SGPRs, where a VOP3 v_fma_f64 reads them directly; as literals every Horner
// step costs a v_mov_b64 first, gfx9 VOP3 taking no 64-bit literal). The kernels get
// it inside their LMConst / as an EKF argument, built on the host by dfmi_trig_k().
struct DfmiTrigK {
  double c[16];  // 2/pi, pi/2 in 3 parts, sin kernel z^5..z^0 coefficients, cos kernel likewise
};
static inline DfmiTrigK dfmi_trig_k(void) {
  DfmiTrigK k = {{6.36619772367581382433e-01, 1.57079632673412561417e+00, 6.07710050630396597660e-11,
                  2.02226624871116645580e-21, 1.58969099521155010221e-10, -2.50507602534068634195e-08,
                  2.75573137070700676789e-06, -1.98412698298579493134e-04, 8.33333333332248946124e-03,
                  -1.66666666666666324348e-01, -1.13596475577881948265e-11, 2.08757232129817482790e-09,
                  -2.75573143513906633035e-07, 2.48015872894767294178e-05, -1.38888888888741095749e-03,
                  4.16666666666666019037e-02}};
  return k;
}

// sincos with the fast path where it is exact to the kernel polynomials' accuracy
// (|x| < 2^19, every argument of these fits) and the library otherwise.
DFMI_HD void dfmi_sincos(double x, double* sn, double* cs) {
  if (fabs(x) < 524288.0) {
    dfmi_sincos_fast(x, sn, cs);
  } else {
#if defined(__HIP_DEVICE_COMPILE__)
    const double2 v = dfmi_sincos_lib(x);
    *sn = v.x;
    *cs = v.y;
#else
    sincos(x, sn, cs);
#endif
  }
}

// dfmi_sincos_k for |r| < pi/4 (no reduction, no quadrant: q = rint(r 2/pi) = 0), same
// bits: the kernel polynomials alone.
DFMI_HD void dfmi_sincos_small(double r, const DfmiTrigK& k, double* sn, double* cs) {
  const double z = r * r;
  const double ps = fma(z, fma(z, fma(z, fma(z, fma(z, k.c[4], k.c[5]), k.c[6]), k.c[7]), k.c[8]), k.c[9]);
  *sn = fma(r * z, ps, r);
  const double pc = fma(z, fma(z, fma(z, fma(z, fma(z, k.c[10], k.c[11]), k.c[12]), k.c[13]), k.c[14]), k.c[15]);
  *cs = fma(z * z, pc, fma(-0.5, z, 1.0));
}

// dfmi_sincos_k(x) with the reduction skipped where it is the identity (|x| < 0.78:
// q = rint(x 2/pi) = 0, r = x), same bits; a wave whose lanes all hold such arguments
// runs the polynomials alone.
DFMI_HD void dfmi_sincos_auto(double x, const DfmiTrigK& k, double* sn, double* cs);

// dfmi_sincos with the constants from k and fewer instructions, same bits: the same
// reduction and Horner polynomials, the quadrant applied as a swap select plus a sign
// flip (no branch, 2 select levels instead of 3), and the library path (|x| >= 2^19, NaN)
// as a rarely taken patch after the fast path instead of an if / else around it. Per-lane
// fp64 chains are issue-bound on gfx950 (a single wave issues a dependent v_fma_f64
// every ~5.4 clocks, as fast as independent ones: profiles/r02l_valu_probe.jsonl), so
// instructions are the cost.
DFMI_HD void dfmi_sincos_k(double x, const DfmiTrigK& k, double* sn, double* cs) {
  const double q = rint(x * k.c[0]);
  double r = fma(-q, k.c[1], x);
  r = fma(-q, k.c[2], r);
  r = fma(-q, k.c[3], r);
  const double z = r * r;
  const double ps = fma(z, fma(z, fma(z, fma(z, fma(z, k.c[4], k.c[5]), k.c[6]), k.c[7]), k.c[8]), k.c[9]);
  const double sr = fma(r * z, ps, r);
  const double pc = fma(z, fma(z, fma(z, fma(z, fma(z, k.c[10], k.c[11]), k.c[12]), k.c[13]), k.c[14]), k.c[15]);
  const double cr = fma(z * z, pc, fma(-0.5, z, 1.0));
  const int qi = ((int)q) & 3;
  const double a = (qi & 1) ? cr : sr;  // sin: sr, cr, -sr, -cr
  const double b = (qi & 1) ? sr : cr;  // cos: cr, -sr, -cr, sr
  *sn = (qi & 2) ? -a : a;
  *cs = ((qi + 1) & 2) ? -b : b;
  if (__builtin_expect(!(fabs(x) < 524288.0), 0)) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double2 v = dfmi_sincos_lib(x);
    *sn = v.x;
    *cs = v.y;
#else
    sincos(x, sn, cs);
#endif
  }
}

DFMI_HD void dfmi_sincos_auto(double x, const DfmiTrigK& k, double* sn, double* cs) {
  if (fabs(x) < 0.78) dfmi_sincos_small(x, k, sn, cs);
  else dfmi_sincos_k(x, k, sn, cs);
}
