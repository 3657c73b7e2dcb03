// lm.h — per-segment Levenberg–Marquardt kernel for gfx950 (fp64).
//
// Reference (file:line in /root/reference):
//   coeffs ................... fit.py:68-150   -> eval_full
//   ssqf ..................... fit.py:152-167  -> eval_ssq
//   msolve ................... fit.py:169-206  -> damped_solve
//   _run_lma_fit ............. fit.py:208-258  -> lm_descend
//   _find_best_initial_guess . fit.py:260-320  -> m_grid_seed
//   fit ...................... fit.py:322-361  -> fit_segment
//   _process_fit_chunk ....... fitters.py:13-60 (warm start inside a chunk) -> lm_chunks_kernel
//
// Mapping: ONE LANE OWNS ONE CHUNK (a run of segments fitted with a warm-start
// chain, np.array_split semantics). With chunk size 1 — the default GPU mode —
// every lane fits one segment, so a wave fits 64 segments at once with no
// shuffles at all; the whole 4-parameter problem (2·ndata residuals, J^T J,
// J^T r, the damped 4×4 solve) lives in that lane's registers. QI is stored
// component-major (qi[c·ld + s]) so the 64 lanes of a wave read each harmonic
// with one coalesced load.
//
// Bessel values come from the two-pass Miller walk in dfmi_math.h, evaluated in
// DESCENDING harmonic order so that no per-lane array is needed; harmonic
// sums are therefore accumulated from j = ndata down to 1 (rounding-level
// difference to the reference's BLAS dot, covered by the parity tolerances).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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
};

// cos(phi + j*pi/2) from (cos phi, sin phi): j mod 4 -> c, -s, -c, s
__host__ __device__ __forceinline__ double quarter_turn(int j, double c, double s) {
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

// Harmonic walk shared by eval_full / eval_ssq: calls body(j, Jm1, J0, Jp1,
// cos(j psi), sin(j psi)) for j = ndata..1.
template <typename Body>
__host__ __device__ __forceinline__ void harmonic_walk(int ndata, double m, double psi, Body&& body) {
  double s1, c1;
  sincos(psi, &s1, &c1);
  double sj, cj;
  sincos((double)ndata * psi, &sj, &cj);
  if (m == 0.0) {  // J_0 = 1, J_k = 0 (k >= 1)
    for (int j = ndata; j >= 1; --j) {
      body(j, j == 1 ? 1.0 : 0.0, 0.0, 0.0, cj, sj);
      const double cn = fma(cj, c1, sj * s1);
      const double sn = fma(sj, c1, -(cj * s1));
      cj = cn;
      sj = sn;
    }
    return;
  }
  const double am = fabs(m);
  if (!(am < 1.0e5)) {  // NaN / absurd m: propagate NaN like scipy would make it useless
    const double nan = __builtin_nan("");
    for (int j = ndata; j >= 1; --j) body(j, nan, nan, nan, cj, sj);
    return;
  }
  if (am < DFMI_BES_TINY) {
    for (int j = ndata; j >= 1; --j) {
      body(j, dfmi_bessel_series(j - 1, m), dfmi_bessel_series(j, m), dfmi_bessel_series(j + 1, m), cj, sj);
      const double cn = fma(cj, c1, sj * s1);
      const double sn = fma(sj, c1, -(cj * s1));
      cj = cn;
      sj = sn;
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
    const double cn = fma(cj, c1, sj * s1);   // cos((j-1) psi)
    const double sn = fma(sj, c1, -(cj * s1));  // sin((j-1) psi)
    cj = cn;
    sj = sn;
  }
}

// fit.py:68-150 (coeffs)
__host__ __device__ __noinline__ void eval_full(const double* __restrict__ q, int64_t ld, int ndata, const double (&p)[4],
                                       Eval& e) {
  const double a = p[0], m = p[1], phi = p[2], psi = p[3];
  double sph, cph;
  sincos(phi, &sph, &cph);
  const bool a_nz = (a != 0.0);
  e = Eval{0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  harmonic_walk(ndata, m, psi, [&](int j, double Jm1, double J0, double Jp1, double cj, double sj) {
    const double pt = quarter_turn(j, cph, sph);       // cos(phi + j pi/2)
    const double ptd = quarter_turn(j + 1, cph, sph);  // cos(phi + j pi/2 + pi/2)
    const double dJ = 0.5 * (Jm1 - Jp1);
    const double common = a * pt * J0;
    const double mq = common * cj;
    const double mi = -common * sj;
    const double rq = q[(int64_t)(j - 1) * ld] - mq;
    const double ri = q[(int64_t)(j - 1 + ndata) * ld] - mi;
    e.ssq = fma(rq, rq, e.ssq);
    e.ssq = fma(ri, ri, e.ssq);
    // rows of J for the Q and I components
    const double q0 = a_nz ? mq / a : 0.0;
    const double i0 = a_nz ? mi / a : 0.0;
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
  });
}

// fit.py:152-167 (ssqf)
__host__ __device__ __noinline__ double eval_ssq(const double* __restrict__ q, int64_t ld, int ndata, const double (&p)[4]) {
  const double a = p[0], m = p[1], phi = p[2], psi = p[3];
  double sph, cph;
  sincos(phi, &sph, &cph);
  double ssq = 0.0;
  harmonic_walk(ndata, m, psi, [&](int j, double, double J0, double, double cj, double sj) {
    const double common = a * quarter_turn(j, cph, sph) * J0;
    const double rq = q[(int64_t)(j - 1) * ld] - common * cj;
    const double ri = q[(int64_t)(j - 1 + ndata) * ld] + common * sj;
    ssq = fma(rq, rq, ssq);
    ssq = fma(ri, ri, ssq);
  });
  return ssq;
}

// fit.py:169-206 (msolve): (JtJ + lam diag(JtJ)) dp = Jt r by LU with partial
// pivoting (LAPACK dgesv semantics: first max |pivot|; an exactly-zero pivot
// is a singular matrix -> LinAlgError in numpy -> dp = 0).
__host__ __device__ __forceinline__ void damped_solve(const Eval& e, double lam, double (&dp)[4]) {
  double A[4][4] = {{e.a00 + lam * e.a00, e.a01, e.a02, e.a03},
                    {e.a01, e.a11 + lam * e.a11, e.a12, e.a13},
                    {e.a02, e.a12, e.a22 + lam * e.a22, e.a23},
                    {e.a03, e.a13, e.a23, e.a33 + lam * e.a33}};
  double b[4] = {e.g0, e.g1, e.g2, e.g3};
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
    // swap rows c and piv (predicated: keep registers static)
#pragma unroll
    for (int r = c + 1; r < 4; ++r) {
      if (r == piv) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const double t = A[c][k];
          A[c][k] = A[r][k];
          A[r][k] = t;
        }
        const double t = b[c];
        b[c] = b[r];
        b[r] = t;
      }
    }
    const double pv = A[c][c];
    if (pv == 0.0) singular = true;
    const double inv = 1.0 / pv;
#pragma unroll
    for (int r = c + 1; r < 4; ++r) {
      const double l = A[r][c] * inv;
#pragma unroll
      for (int k = c + 1; k < 4; ++k) A[r][k] = fma(-l, A[c][k], A[r][k]);
      b[r] = fma(-l, b[c], b[r]);
    }
  }
  if (singular) {
    dp[0] = dp[1] = dp[2] = dp[3] = 0.0;
    return;
  }
#pragma unroll
  for (int r = 3; r >= 0; --r) {
    double s = b[r];
#pragma unroll
    for (int k = r + 1; k < 4; ++k) s = fma(-A[r][k], dp[k], s);
    dp[r] = s / A[r][r];
  }
}

__host__ __device__ __forceinline__ double norm4(double a, double b, double c, double d) {
  return sqrt(a * a + b * b + c * c + d * d);
}

// fit.py:208-258 (_run_lma_fit). p in/out; returns ssq0 at the final p.
__host__ __device__ double lm_descend(const double* __restrict__ q, int64_t ld, int ndata, double (&p)[4], const LMConst& c) {
  Eval e;
  eval_full(q, ld, ndata, p, e);
  for (int it = 0; it < c.max_steps; ++it) {
    const double po[4] = {p[0], p[1], p[2], p[3]};
    bool found = false;
    double best_ssq = e.ssq;
    double pt[4];
    for (int li = 0; li < c.n_lambda; ++li) {
      double dp[4];
      damped_solve(e, c.lambdas[li], dp);
      if (norm4(dp[0], dp[1], dp[2], dp[3]) < c.min_step_norm) continue;
      pt[0] = p[0] + dp[0];
      pt[1] = p[1] + dp[1];
      pt[2] = p[2] + dp[2];
      pt[3] = p[3] + dp[3];
      const double s = eval_ssq(q, ld, ndata, pt);
      if (s < best_ssq) {
        best_ssq = s;
        found = true;
        break;
      }
    }
    if (!found) break;
    p[0] = pt[0];
    p[1] = pt[1];
    p[2] = pt[2];
    p[3] = pt[3];
    eval_full(q, ld, ndata, p, e);
    const double change = norm4(p[0] - po[0], p[1] - po[1], p[2] - po[2], p[3] - po[3]);
    if ((e.ssq - best_ssq) < c.conv_improve && change < c.conv_param_change) break;
  }
  return e.ssq;
}

// ssq at a grid point (psi = 0 exactly: cos(j*0)=1, sin(j*0)=0), Bessel values
// J_j(mtry) from the host-built table.
__host__ __device__ double grid_ssq(const double* __restrict__ q, int64_t ld, int ndata, const double* __restrict__ jrow,
                           double a, double phi) {
  double sph, cph;
  sincos(phi, &sph, &cph);
  double ssq = 0.0;
  for (int j = 1; j <= ndata; ++j) {
    const double common = a * quarter_turn(j, cph, sph) * jrow[j - 1];
    const double rq = q[(int64_t)(j - 1) * ld] - common;
    const double ri = q[(int64_t)(j - 1 + ndata) * ld] + common * 0.0;
    ssq = fma(rq, rq, ssq);
    ssq = fma(ri, ri, ssq);
  }
  return ssq;
}

// fit.py:260-320 (_find_best_initial_guess). jtab: n_grid rows of J_1..J_ndata.
__host__ __device__ void m_grid_seed(const double* __restrict__ q, int64_t ld, int ndata, const double* __restrict__ jtab,
                            const LMConst& c, double (&best)[4]) {
  double best_ssq = 9e99;
  best[0] = best[1] = best[2] = best[3] = 0.0;
  for (int g = 0; g < c.n_grid; ++g) {
    const double mtry = c.grid_min + (double)g * c.grid_delta;
    const double* jrow = jtab + (int64_t)g * ndata;
    double sinsum = 0.0, cossum = 0.0;
    int nsin = 0, ncos = 0;
    for (int i = 0; i < ndata; ++i) {
      const int j = i + 1;
      const double bq = jrow[i] * 1.0;   // jv * cos(j*0)
      const double bi = jrow[i] * -0.0;  // jv * -sin(j*0)
      const double dq = q[(int64_t)i * ld], di = q[(int64_t)(i + ndata) * ld];
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
    if (nsin == 0 || ncos == 0) continue;
    const double ptry = atan2(sinsum / (double)nsin, cossum / (double)ncos);
    double sp, cp;
    sincos(ptry, &sp, &cp);
    const double tab4[4] = {cp, -sp, -cp, sp};
    double asum = 0.0;
    int na = 0;
    for (int i = 0; i < ndata; ++i) {
      const int j = i + 1;
      const double sc = tab4[j & 3];
      const double bq = jrow[i] * 1.0;
      const double bi = jrow[i] * -0.0;
      if (fabs(bq) > c.bessel_amp_thr && fabs(sc) > c.sincos_amp_thr) {
        asum += q[(int64_t)i * ld] / (sc * bq);
        ++na;
      }
      if (fabs(bi) > c.bessel_amp_thr && fabs(sc) > c.sincos_amp_thr) {
        asum += q[(int64_t)(i + ndata) * ld] / (sc * bi);
        ++na;
      }
    }
    if (na == 0) continue;
    const double atry = asum / (double)na;
    const double s = grid_ssq(q, ld, ndata, jrow, atry, ptry);
    if (s < best_ssq) {
      best_ssq = s;
      best[0] = atry;
      best[1] = mtry;
      best[2] = ptry;
      best[3] = 0.0;
    }
  }
}

// fit.py:322-361 (fit): LM, status + grid retry, normalisation, phi wrap.
__host__ __device__ int fit_segment(const double* __restrict__ q, int64_t ld, int ndata, const double* __restrict__ jtab,
                           const LMConst& c, double (&p)[4], double& ssq_out) {
  double ssq = lm_descend(q, ld, ndata, p, c);
  int status;
  if (ssq < c.fitok_threshold) {
    status = 0;
  } else {
    double g[4];
    m_grid_seed(q, ld, ndata, jtab, c, g);
    if (!(g[0] == 0.0) || !(g[1] == 0.0) || !(g[2] == 0.0) || !(g[3] == 0.0)) {  // np.any
      const double ssq2 = lm_descend(q, ld, ndata, g, c);
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

// Guess source for record r, component i: guess[r*g_rec + i*g_comp].
struct GuessInline {
  double v[8][4];
};

// One lane per chunk. Records r < nrec each hold nbuf segments; the fitted
// items of record r are segments [first, first + nitems); they are cut into
// nchunk chunks with np.array_split semantics and each chunk starts from the
// record's guess, warm-starting within the chunk (fitters.py:42-58).
__global__ __launch_bounds__(256) void lm_chunks_kernel(
    const double* __restrict__ qi, int64_t qi_ld, int ndata, int64_t nrec, int64_t nbuf, int64_t first,
    int64_t nitems, int64_t nchunk, const double* __restrict__ guess, int64_t g_rec, int64_t g_comp,
    GuessInline ginl, int use_inline, const double* __restrict__ jtab, LMConst c, double* __restrict__ out,
    int64_t out_ld, int32_t* __restrict__ status) {
  const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (id >= nrec * nchunk) return;
  const int64_t r = id / nchunk;
  const int64_t k = id - r * nchunk;
  const int64_t qn = nitems / nchunk, rm = nitems % nchunk;
  const int64_t start = k * qn + (k < rm ? k : rm);
  const int64_t len = qn + (k < rm ? 1 : 0);
  double p[4];
  if (use_inline) {
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = ginl.v[r][i];
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = guess[r * g_rec + i * g_comp];
  }
  for (int64_t t = 0; t < len; ++t) {
    const int64_t sidx = r * nbuf + first + start + t;
    double ssq;
    const int st = fit_segment(qi + sidx, qi_ld, ndata, jtab, c, p, ssq);
    out[0 * out_ld + sidx] = p[0];
    out[1 * out_ld + sidx] = p[1];
    out[2 * out_ld + sidx] = p[2];
    out[3 * out_ld + sidx] = p[3];
    out[5 * out_ld + sidx] = ssq;
    status[sidx] = st;
  }
}

}  // namespace dfmi
