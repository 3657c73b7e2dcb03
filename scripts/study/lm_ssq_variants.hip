// Evaluation variants of ssqf for scripts/study/lm_ssq_noise.py (study only).
#include "../../deepfmkit_amd/csrc/dfmi_math.h"
#include "../../deepfmkit_amd/csrc/lm.h"
extern "C" void var_ssq(const double* qi, const double* p, long n, int jsrc, int tpsi, int tphi, int acc, double* out) {
  const DfmiTrigK k = dfmi_trig_k();
  for (long i = 0; i < n; ++i) {
    const double a = p[4*i], m = p[4*i+1], phi = p[4*i+2], psi = p[4*i+3];
    double J[14];
    if (jsrc == 0) dfmi::bessel_regs<14>(m, 11, J);
    else { double t[14]; dfmi_bessel_table(m, 13, t); for (int q = 0; q < 14; ++q) J[q] = t[q]; }
    double sph, cph, s1, c1;
    if (tphi == 0) dfmi_sincos_auto(phi, k, &sph, &cph); else sincos(phi, &sph, &cph);
    if (tphi == 0) dfmi_sincos_auto(psi, k, &s1, &c1); else sincos(psi, &s1, &c1);
    double cjs[11], sjs[11];
    if (tpsi == 0) {
      double cj = c1, sj = s1, cm = 1.0, sm = 0.0, tc = 2.0 * c1;
      for (int j = 1; j <= 10; ++j) { cjs[j] = cj; sjs[j] = sj; double cn = fma(tc, cj, -cm), sn = fma(tc, sj, -sm); cm = cj; sm = sj; cj = cn; sj = sn; }
    } else if (tpsi == 1) {
      double sj, cj; sincos(10.0 * psi, &sj, &cj);
      for (int j = 10; j >= 1; --j) { cjs[j] = cj; sjs[j] = sj; double cn = fma(cj, c1, sj * s1), sn = fma(sj, c1, -(cj * s1)); cj = cn; sj = sn; }
    } else if (tpsi == 3) {
      double cj = c1, sj = s1;
      for (int j = 1; j <= 10; ++j) { cjs[j] = cj; sjs[j] = sj; double cn = fma(cj, c1, -(sj * s1)), sn = fma(sj, c1, cj * s1); cj = cn; sj = sn; }
    } else if (tpsi == 4) {  // Reinsch: alpha = 1 - cos psi = 2 sin^2(psi/2)
      double sh, ch; sincos(0.5 * psi, &sh, &ch); const double al = 2.0 * sh * sh;
      double cj = c1, sj = s1, dc = c1 - 1.0, ds = s1;  // dc = cos(psi) - cos(0)
      dc = -al; 
      for (int j = 1; j <= 10; ++j) { cjs[j] = cj; sjs[j] = sj; dc = fma(-2.0 * al, cj, dc); ds = fma(-2.0 * al, sj, ds); cj += dc; sj += ds; }
    } else {
      for (int j = 1; j <= 10; ++j) sincos(j * psi, &sjs[j], &cjs[j]);
    }
    double so = 0, se = 0;
    const double ac = a * cph, as = a * sph;
    for (int j = 1; j <= 10; ++j) {
      double c = (acc == 0) ? dfmi::quarter_turn(j, ac, as) * J[j] : a * dfmi::quarter_turn(j, cph, sph) * J[j];
      double rq = fma(-c, cjs[j], qi[j-1]);
      double ri = fma(c, sjs[j], qi[j+9]);
      double& s = (j & 1) ? so : se;
      s = fma(rq, rq, s); s = fma(ri, ri, s);
    }
    out[i] = so + se;
  }
}
