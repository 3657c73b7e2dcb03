/* ekf_scalar.c — TEST / BASELINE INFRASTRUCTURE (never linked into libdfmi.so).
 *
 * Scalar C restatement of EKFFitter.fit's per-sample loop (reference
 * fitters.py:274-302) in the operation order of the numpy expressions, as the
 * oracle (oracle/nls_oracle.py ekf_record) states them: P = F P F^T + Q (F = I),
 * theta = w_m t_k + psi, H, S = H P H^T + R, K = (P H^T) inv(S), x += K y,
 * P = (I - K H) P (full 5x5 products). The CPU "host scalar loop" baseline of
 * SURVEY.md §8(d) for config 5: one channel on one core, libm sin / cos.
 * Built by oracle/Makefile into oracle/libekf_scalar.so (ctypes: scripts/bench_ekf.py,
 * tests/test_oracle_c.py). x0[5] = (a, m, phi, psi, dc), states: nbuf x 5.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

void ekf_scalar(const double* x, int64_t n, const double* x0, const double* p0_diag, const double* q_diag,
                double r_val, double w_m, double f_samp, int64_t R, int64_t nbuf, double* states) {
  double st[5], P[5][5], Q[5];
  memcpy(st, x0, sizeof(st));
  for (int i = 0; i < 5; ++i) {
    Q[i] = q_diag[i];
    for (int j = 0; j < 5; ++j) P[i][j] = (i == j) ? p0_diag[i] : 0.0;
  }
  for (int64_t k = 0; k < n; ++k) {
    for (int i = 0; i < 5; ++i) P[i][i] += Q[i];
    const double a = st[0], m = st[1], phi = st[2], psi = st[3], dc = st[4];
    const double t = (double)k / f_samp;
    const double th = w_m * t + psi;
    const double cth = cos(th), sth = sin(th);
    const double arg = phi + m * cth;
    const double ca = cos(arg), sa = sin(arg);
    const double h = a * ca + dc;
    const double H[5] = {ca, -a * sa * cth, -a * sa, a * m * sa * sth, 1.0};
    const double y = x[k] - h;
    double HP[5], PH[5];
    for (int j = 0; j < 5; ++j) {
      double s = 0.0, u = 0.0;
      for (int i = 0; i < 5; ++i) {
        s += H[i] * P[i][j];
        u += P[j][i] * H[i];
      }
      HP[j] = s;
      PH[j] = u;
    }
    double S = 0.0;
    for (int j = 0; j < 5; ++j) S += HP[j] * H[j];
    S += r_val;
    const double invS = 1.0 / S;
    double K[5];
    for (int i = 0; i < 5; ++i) {
      K[i] = PH[i] * invS;
      st[i] += K[i] * y;
    }
    double Pn[5][5];
    for (int i = 0; i < 5; ++i)
      for (int j = 0; j < 5; ++j) {
        double s = 0.0;
        for (int l = 0; l < 5; ++l) s += ((i == l ? 1.0 : 0.0) - K[i] * H[l]) * P[l][j];
        Pn[i][j] = s;
      }
    memcpy(P, Pn, sizeof(P));
    if ((k + 1) % R == 0) {
      const int64_t b = (k + 1) / R - 1;
      if (b < nbuf) memcpy(states + b * 5, st, sizeof(st));
    }
  }
}
