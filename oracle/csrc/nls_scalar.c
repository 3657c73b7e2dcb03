/* nls_scalar.c — TEST / BASELINE INFRASTRUCTURE ONLY (never linked into the product).
 *
 * A scalar C restatement of the reference's per-segment NLS readout, for bench.py's
 * second CPU baseline ("an optional second baseline is a C++ scalar
 * restatement, OpenMP, same cores"): _fit_parallel with chunk size 1 (fitters.py:395-428:
 * buffer 0 fitted from the guess, every other buffer from its result), each buffer
 *   calculate_quadratures + mean    fit.py:18-66, fitters.py:45-49 (the basis cos/sin of
 *                                   fl(fl(h w0) t), as numpy forms the angle, computed
 *                                   once per call instead of once per buffer; plain
 *                                   sequential sums: not numpy's pairwise order)
 *   coeffs / ssqf / msolve          fit.py:68-206 (4x4 LU with partial pivoting,
 *                                   exactly-zero pivot -> dp = 0)
 *   _run_lma_fit                    fit.py:208-258
 *   _find_best_initial_guess        fit.py:260-320
 *   fit                             fit.py:322-361
 * with J_0..J_{ndata+1}(m) from one Miller recurrence per evaluation (the reference
 * calls scipy.special.jv per order), the quadratures by folding the buffer into the
 * basis period's phase bins first where the period divides R (the reference multiplies
 * 2 ndata full-length trig arrays). Buffers are distributed over OpenMP threads. Not bit-exact with the reference (summation order,
 * Bessel routine): it is a speed baseline, checked against the numpy oracle at 1e-9 on
 * status-0 buffers (tests/test_oracle_c.py).
 */
#define _DEFAULT_SOURCE /* M_PI */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NDMAX 64

/* J_0..J_n(x) (n <= NDMAX + 1) by one backward Miller recurrence normalised with
 * J_0 + 2 sum J_2k = 1 (start order as dfmi_bessel_start), J_k(-x) = (-1)^k J_k(x). */
static void bessel_all(double x, int n, double* J) {
  const double ax = fabs(x);
  if (ax < 1e-300) {
    for (int k = 0; k <= n; ++k) J[k] = k == 0 ? 1.0 : 0.0;
    return;
  }
  int M = (int)(1.1 * ax + 14.0 + 3.0 * sqrt(ax)) + 1;
  if (M < n + 10) M = n + 10;
  M = (M + 1) & ~1;
  const double tox = 2.0 / ax;
  double fp1 = 0.0, f = 1.0, S = 2.0;
  for (int k = M; k >= 1; --k) {
    double fm1 = (double)k * tox * f - fp1;
    if (fabs(fm1) > 1e250) {
      fm1 *= 1e-250;
      f *= 1e-250;
      S *= 1e-250;
      for (int i = k; i <= n && i <= M; ++i) J[i] *= 1e-250;
    }
    if (k - 1 <= n) J[k - 1] = fm1;
    if (k == M && k <= n) J[k] = f;
    if (k - 1 == 0) S += fm1;
    else if (((k - 1) & 1) == 0) S += 2.0 * fm1;
    fp1 = f;
    f = fm1;
  }
  for (int k = 0; k <= n; ++k) J[k] = J[k] / S * ((x < 0 && (k & 1)) ? -1.0 : 1.0);
}

static const double kLadder[8] = {0.0, 1e-7, 1e-5, 1e-3, 1e-1, 1.0, 10.0, 100.0};

typedef struct {
  double ssq, jtj[16], g[4];
} Eval;

static void coeffs(int nd, const double* qi, const double* p, Eval* e) {
  const double a = p[0], m = p[1], phi = p[2], psi = p[3];
  double J[4 * 2 * NDMAX];
  double r[2 * NDMAX];
  double B[NDMAX + 2];
  bessel_all(m, nd + 1, B);
  memset(J, 0, sizeof(double) * 8 * nd);
  double ssq = 0.0;
  for (int k = 0; k < nd; ++k) {
    const int j = k + 1;
    const double pt = cos(phi + j * M_PI / 2.0);
    const double cj = cos(j * psi), sj = sin(j * psi);
    const double bj = B[j];
    const double dbj = 0.5 * (B[j - 1] - B[j + 1]);
    const double common = a * pt * bj;
    const double mq = common * cj, mi = -common * sj;
    r[k] = qi[k] - mq;
    r[nd + k] = qi[nd + k] - mi;
    if (a != 0.0) {
      J[k * 4 + 0] = mq / a;
      J[(nd + k) * 4 + 0] = mi / a;
    }
    const double cm = a * pt * dbj;
    J[k * 4 + 1] = cm * cj;
    J[(nd + k) * 4 + 1] = -cm * sj;
    const double cphi = a * cos(phi + j * M_PI / 2.0 + M_PI / 2.0) * bj;
    J[k * 4 + 2] = cphi * cj;
    J[(nd + k) * 4 + 2] = -cphi * sj;
    J[k * 4 + 3] = common * -sj * j;
    J[(nd + k) * 4 + 3] = -common * cj * j;
  }
  for (int i = 0; i < 2 * nd; ++i) ssq += r[i] * r[i];
  e->ssq = ssq;
  for (int u = 0; u < 4; ++u) {
    double gu = 0.0;
    for (int i = 0; i < 2 * nd; ++i) gu += J[i * 4 + u] * r[i];
    e->g[u] = gu;
    for (int v = 0; v < 4; ++v) {
      double s = 0.0;
      for (int i = 0; i < 2 * nd; ++i) s += J[i * 4 + u] * J[i * 4 + v];
      e->jtj[u * 4 + v] = s;
    }
  }
}

static double ssqf(int nd, const double* qi, const double* p) {
  const double a = p[0], m = p[1], phi = p[2], psi = p[3];
  double B[NDMAX + 2];
  bessel_all(m, nd, B);
  double s = 0.0;
  for (int k = 0; k < nd; ++k) {
    const int j = k + 1;
    const double common = a * cos(phi + j * M_PI / 2.0) * B[j];
    const double rq = qi[k] - common * cos(j * psi);
    const double ri = qi[nd + k] + common * sin(j * psi);
    s += rq * rq + ri * ri;
  }
  return s;
}

static void msolve(double lam, const double* jtj, const double* g, double* dp) {
  double A[4][5];
  for (int i = 0; i < 4; ++i) {
    for (int j = 0; j < 4; ++j) A[i][j] = jtj[i * 4 + j] + (i == j ? lam * jtj[i * 4 + j] : 0.0);
    A[i][4] = g[i];
  }
  for (int c = 0; c < 4; ++c) {
    int piv = c;
    for (int i = c + 1; i < 4; ++i)
      if (fabs(A[i][c]) > fabs(A[piv][c])) piv = i;
    if (A[piv][c] == 0.0) {
      dp[0] = dp[1] = dp[2] = dp[3] = 0.0;
      return;
    }
    if (piv != c)
      for (int j = 0; j < 5; ++j) {
        const double t = A[c][j];
        A[c][j] = A[piv][j];
        A[piv][j] = t;
      }
    for (int i = c + 1; i < 4; ++i) {
      const double f = A[i][c] / A[c][c];
      for (int j = c; j < 5; ++j) A[i][j] -= f * A[c][j];
    }
  }
  for (int i = 3; i >= 0; --i) {
    double s = A[i][4];
    for (int j = i + 1; j < 4; ++j) s -= A[i][j] * dp[j];
    dp[i] = s / A[i][i];
  }
}

static double lm_descend(int nd, const double* qi, double* p) {
  Eval e;
  coeffs(nd, qi, p, &e);
  for (int it = 0; it < 100; ++it) {
    double pp[4], best = e.ssq, bp[4];
    memcpy(pp, p, sizeof pp);
    memcpy(bp, p, sizeof bp);
    for (int l = 0; l < 8; ++l) {
      double dp[4];
      msolve(kLadder[l], e.jtj, e.g, dp);
      if (sqrt(dp[0] * dp[0] + dp[1] * dp[1] + dp[2] * dp[2] + dp[3] * dp[3]) < 1e-15) continue;
      double t[4] = {p[0] + dp[0], p[1] + dp[1], p[2] + dp[2], p[3] + dp[3]};
      const double s = ssqf(nd, qi, t);
      if (s < best) {
        best = s;
        memcpy(bp, t, sizeof bp);
        break;
      }
    }
    if (best >= e.ssq) break;
    memcpy(p, bp, sizeof bp);
    coeffs(nd, qi, p, &e);
    const double d0 = p[0] - pp[0], d1 = p[1] - pp[1], d2 = p[2] - pp[2], d3 = p[3] - pp[3];
    if ((e.ssq - best) < 1e-9 && sqrt(d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3) < 1e-9) break;
  }
  return e.ssq;
}

static void m_grid_seed(int nd, const double* qi, double* best_p) {
  double best = 9e99;
  best_p[0] = best_p[1] = best_p[2] = best_p[3] = 0.0;
  for (int gi = 0; gi <= 50; ++gi) {
    const double mtry = 5.0 + 0.5 * gi;
    double Bg[NDMAX + 2];
    bessel_all(mtry, nd, Bg);
    double ssum = 0.0, csum = 0.0;
    int ns = 0, nc = 0;
    for (int k = 0; k < nd; ++k) {
      const int j = k + 1;
      const double bes = Bg[j];
      const double bq = bes, bi = bes * -0.0;
      const double dq = qi[k], di = qi[nd + k];
      for (int w = 0; w < 2; ++w) {
        const double data = w ? di : dq, b = w ? bi : bq;
        if (fabs(b) > 0.05) {
          switch (j % 4) {
            case 0: csum += data / b; ++nc; break;
            case 1: ssum -= data / b; ++ns; break;
            case 2: csum -= data / b; ++nc; break;
            default: ssum += data / b; ++ns; break;
          }
        }
      }
    }
    if (ns == 0 || nc == 0) continue;
    const double ptry = atan2(ssum / ns, csum / nc);
    const double tab[4] = {cos(ptry), -sin(ptry), -cos(ptry), sin(ptry)};
    double asum = 0.0;
    int na = 0;
    for (int k = 0; k < nd; ++k) {
      const int j = k + 1;
      const double sc = tab[j % 4];
      const double bes = Bg[j];
      const double bq = bes, bi = bes * -0.0;
      const double dq = qi[k], di = qi[nd + k];
      for (int w = 0; w < 2; ++w) {
        const double data = w ? di : dq, b = w ? bi : bq;
        if (fabs(b) > 0.05 && fabs(sc) > 0.1) {
          asum += data / (sc * b);
          ++na;
        }
      }
    }
    if (na == 0) continue;
    const double trial[4] = {asum / na, mtry, ptry, 0.0};
    const double s = ssqf(nd, qi, trial);
    if (s < best) {
      best = s;
      memcpy(best_p, trial, sizeof trial);
    }
  }
}

static int fit_segment(int nd, const double* qi, double* p, double* ssq_out) {
  double ssq = lm_descend(nd, qi, p);
  int status;
  if (ssq < 1e-3) {
    status = 0;
  } else {
    double g[4];
    m_grid_seed(nd, qi, g);
    if (g[0] != 0.0 || g[1] != 0.0 || g[2] != 0.0 || g[3] != 0.0) {
      const double s2 = lm_descend(nd, qi, g);
      if (s2 < ssq) {
        ssq = s2;
        memcpy(p, g, sizeof g);
      }
    }
    status = ssq < 1e-3 ? 1 : 2;
  }
  if (p[0] < 0) {
    p[0] = -p[0];
    p[2] += M_PI;
  }
  if (p[1] < 0) {
    p[1] = -p[1];
    p[2] += M_PI;
  }
  const double twopi = 2.0 * M_PI;
  double r = fmod(p[2] + M_PI, twopi);  /* Python float %: the sign of the divisor */
  if (r != 0.0 && r < 0.0) r += twopi;
  p[2] = r - M_PI;
  *ssq_out = ssq;
  return status;
}

/* tab: [L][2 nd] (t-major) over one period L of the basis when L > 0 (the samples are
 * folded into L phase bins first: sum_t x_t b(t) = sum_p b(p) sum_k x_{p + kL}), else
 * over all R samples. */
static void demod(const double* x, int R, int L, int nd, const double* tab, double* qi, double* dc) {
  double acc[2 * NDMAX];
  for (int h = 0; h < 2 * nd; ++h) acc[h] = 0.0;
  double sdc = 0.0;
  if (L > 0) {
    double bins[4096];
    for (int p = 0; p < L; ++p) bins[p] = x[p];
    for (int t0 = L; t0 < R; t0 += L)
      for (int p = 0; p < L; ++p) bins[p] += x[t0 + p];
    for (int p = 0; p < L; ++p) {
      const double v = bins[p];
      const double* b = tab + (size_t)p * 2 * nd;
      for (int h = 0; h < 2 * nd; ++h) acc[h] += v * b[h];
      sdc += v;
    }
  } else {
    for (int t = 0; t < R; ++t) {
      const double v = x[t];
      const double* b = tab + (size_t)t * 2 * nd;
      for (int h = 0; h < 2 * nd; ++h) acc[h] += v * b[h];
      sdc += v;
    }
  }
  for (int h = 0; h < 2 * nd; ++h) qi[h] = acc[h] / R;
  *dc = sdc / R;
}

static void fit_buffer(const double* x, int R, int L, int nd, const double* tab, const double* guess, double* row) {
  double qi[2 * NDMAX], dc, p[4] = {guess[0], guess[1], guess[2], guess[3]}, ssq;
  demod(x, R, L, nd, tab, qi, &dc);
  const int st = fit_segment(nd, qi, p, &ssq);
  row[0] = p[0];
  row[1] = p[1];
  row[2] = p[2];
  row[3] = p[3];
  row[4] = dc;
  row[5] = ssq;
  row[6] = st;
}

/* out: nbuf x 7 (amp, m, phi, psi, dc, ssq, fitok). Returns 0, or -1 on bad arguments. */
int nls_scalar_record(const double* x, int64_t nbuf, int R, int nd, double w0, const double* guess, int nthreads,
                      double* out) {
  if (nbuf < 1 || R < 1 || nd < 1 || nd > NDMAX) return -1;
  /* the basis period: L samples with L w0 a whole number of turns (to 1e-9 rad) dividing R */
  int L = 0;
  for (int c = 1; c <= 64 && !L; ++c) {
    const double l = 2.0 * M_PI * c / w0;
    const int li = (int)floor(l + 0.5);
    if (li > 0 && li <= 4096 && fabs(li * w0 - 2.0 * M_PI * c) < 1e-9 && R % li == 0) L = li;
  }
  const int T = L > 0 ? L : R;
  double* tab = (double*)malloc(sizeof(double) * 2 * nd * (size_t)T);
  if (!tab) return -1;
  for (int t = 0; t < T; ++t)
    for (int h = 0; h < nd; ++h) {
      const double ang = ((h + 1) * w0) * t;
      tab[(size_t)t * 2 * nd + h] = cos(ang);
      tab[(size_t)t * 2 * nd + nd + h] = sin(ang);
    }
  fit_buffer(x, R, L, nd, tab, guess, out);
  const double seed[4] = {out[0], out[1], out[2], out[3]};
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
  for (int64_t b = 1; b < nbuf; ++b) fit_buffer(x + b * (int64_t)R, R, L, nd, tab, seed, out + b * 7);
  free(tab);
  return 0;
}

/* fit.fit (fit.py:322-361) on n QI vectors: qi n x 2 nd (row-major [Q_1..Q_nd, I_1..I_nd]),
 * guess n x 4; out n x 6 (amp, m, phi, psi, ssq, status). Returns 0, or -1. */
int lm_scalar_fit(const double* qi, int64_t n, int nd, const double* guess, int nthreads, double* out) {
  if (n < 0 || nd < 1 || nd > NDMAX) return -1;
#pragma omp parallel for schedule(dynamic, 64) num_threads(nthreads)
  for (int64_t s = 0; s < n; ++s) {
    double p[4] = {guess[s * 4], guess[s * 4 + 1], guess[s * 4 + 2], guess[s * 4 + 3]}, ssq;
    const int st = fit_segment(nd, qi + s * 2 * nd, p, &ssq);
    for (int i = 0; i < 4; ++i) out[s * 6 + i] = p[i];
    out[s * 6 + 4] = ssq;
    out[s * 6 + 5] = st;
  }
  return 0;
}
