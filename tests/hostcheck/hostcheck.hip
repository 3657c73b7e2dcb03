// hostcheck.hip — TEST-ONLY host build of the product's fp64 numerics.
//
// Compiles deepfmkit_amd/csrc/dfmi_math.h and lm.h (whose numerics are
// __host__ __device__) for the CPU so the CPU test suite can check the Bessel
// walk and the per-segment LM against the golden vectors without a GPU; also
// the EKF parallel-in-time stop rule (ekf_pit.h pit_decide). The
// product library never links this; the GPU parity tests (tests/test_gpu_*.py)
// exercise the real kernels.
#include <vector>
#include "../../deepfmkit_amd/csrc/dfmi_math.h"
#include "../../deepfmkit_amd/csrc/lm.h"
#include "../../deepfmkit_amd/csrc/np_sum.h"
#include "../../deepfmkit_amd/csrc/synth.h"
#include "../../deepfmkit_amd/csrc/ekf_pit.h"
#include "../../deepfmkit_amd/csrc/fork_guard.h"

namespace {
struct HKey {
  uint32_t* p;
  uint32_t& operator()(int i) const { return p[i]; }
};
struct HVec {
  double* p;
  double& operator()(int64_t k) const { return p[k]; }
};
}  // namespace

extern "C" {

// fork_guard.h: the message libdfmi.so returns (DFMI_ERR_HIP) to a process forked after
// it initialised HIP; "" when `cur_pid` may call in. Returns the message length.
int hc_fork_guard(long init_pid, long cur_pid, char* buf, int cap) {
  const std::string m = dfmi_fork_guard(init_pid, cur_pid);
  snprintf(buf, cap, "%s", m.c_str());
  return (int)m.size();
}

// numpy summation order (np_sum.h): the plan the W-DFMI kernels run for their means.
double hc_np_sum(const double* a, int n) { return dfmi_plan_sum_host(a, n); }

// synth.h on the host: n gaussians of RandomState(seed) (legacy normal, scale 1)
void hc_mt_gauss(uint32_t seed, int64_t n, double* out) {
  std::vector<uint32_t> key(dfmi::kMtN);
  dfmi::Mt<HKey> mt{HKey{key.data()}, 0, false, 0.0};
  mt.seed(seed);
  for (int64_t k = 0; k < n; ++k) out[k] = mt.next_gauss();
}

// synth.h's whole trial on the host (host libm cos / sin / log)
void hc_synth_trial(const dfmi_synth_trial* p, int64_t n, double f_samp, double* out) {
  std::vector<uint32_t> key(dfmi::kMtN);
  std::vector<double> a(n), d(n), ph(n);
  dfmi::synth_trial(*p, n, f_samp, HKey{key.data()}, HVec{a.data()}, HVec{d.data()}, HVec{ph.data()}, HVec{out});
}

void hc_bessel_table(double x, int N, double* out) { dfmi_bessel_table(x, N, out); }

// layout check of the trial table (physics.SYNTH_TRIAL_DTYPE mirrors dfmi_synth_trial)
int64_t hc_sizeof_synth_trial(void) { return (int64_t)sizeof(dfmi_synth_trial); }

// synth.h's waveform g(tp) for sample k of a trial (before the max-normalisation)
void hc_synth_g(const dfmi_synth_trial* p, int64_t n, double f_samp, double* out) {
  for (int64_t k = 0; k < n; ++k) out[k] = dfmi::synth_g(*p, k, f_samp);
}

// dfmi_pymod (numpy / Python float modulo, the phi wrap of fit.py:357) elementwise
void hc_pymod(const double* a, int64_t n, double b, double* out) {
  for (int64_t k = 0; k < n; ++k) out[k] = dfmi_pymod(a[k], b);
}

// the LM register path's single Miller pass (lm.h bessel_regs): NB = 14 (ndata <= 12)
// or 18 (ndata <= 16), J_0..J_{NB-1}
void hc_bessel_regs(double x, int nb, double* out) {
  if (nb == 14) {
    double J[14];
    dfmi::bessel_regs<14>(x, 13, J);
    for (int k = 0; k < 14; ++k) out[k] = J[k];
  } else {
    double J[18];
    dfmi::bessel_regs<18>(x, 17, J);
    for (int k = 0; k < 18; ++k) out[k] = J[k];
  }
}

// ssqf (fit.py:152-167) of the register path's trial evaluation (reg = 1) or of the literal
// general path (reg = 0) at n points p (n x 4) for ONE segment's QI (2 ndata values)
void hc_ssq_points(const double* qi, int ndata, const double* p, long n, int reg, double* out) {
  const dfmi::QGlobal qg{qi, 1, ndata};
  const DfmiTrigK k = dfmi_trig_k();
  for (long i = 0; i < n; ++i) {
    double pp[4] = {p[4 * i], p[4 * i + 1], p[4 * i + 2], p[4 * i + 3]};
    if (reg && ndata == 10) {
      dfmi::TrialReg<dfmi::kExactNd | 10> t;
      out[i] = dfmi::eval_reg_trial<dfmi::kExactNd | 10>(qg, ndata, pp, t, k);
    } else {
      dfmi::Eval e;
      dfmi::eval_gen(qg, ndata, pp, e);
      out[i] = e.ssq;
    }
  }
}

// ekf_pit.h's stop rule fed a channel's move sequence (moves[0] is pass 0's, ignored as the
// device ignores it): the pass after which the status left 0 (0: never) and that status.
void hc_pit_decide(const double* moves, int n, double tol, int stall_max, int cap, int* passes_out,
                   int* status_out) {
  dfmi::PitChan c{};
  c.dprev = __builtin_nan("");
  c.rho = -1.0;
  for (int i = 0; i < dfmi::kPitTrend; ++i) c.dold[i] = __builtin_nan("");
  dfmi::PitRule ru{};
  ru.tol = tol;
  ru.noise = tol;
  ru.stall_max = stall_max;
  ru.cap = cap;
  ru.slow_from = 16;
  *passes_out = 0;
  *status_out = 0;
  for (int k = 0; k < n && k < cap; ++k) {
    dfmi::pit_decide(c, moves[k], ru, nullptr);
    if (c.status) {
      *passes_out = c.passes;
      *status_out = c.status;
      return;
    }
  }
}

// qi component-major (qi[c*n + s]); guess n x 4; constants in the reference order.
int hc_fit_segments(const double* qi, long n, int ndata, const double* guess, const double* consts,
                    const double* lambdas, int n_lambda, double* p_out, double* ssq_out, int* status_out,
                    int force_general) {
  dfmi::LMConst c{};
  c.max_steps = (int)consts[0];
  c.conv_improve = consts[1];
  c.conv_param_change = consts[2];
  c.fitok_threshold = consts[3];
  const double gmin = consts[4], gmax = consts[5], gstep = consts[6];
  c.bessel_amp_thr = consts[7];
  c.sincos_amp_thr = consts[8];
  c.min_step_norm = consts[9];
  c.n_lambda = n_lambda;
  for (int i = 0; i < n_lambda; ++i) c.lambdas[i] = lambdas[i];
  const double stop = gmax + gstep;
  const double len = ceil((stop - gmin) / gstep);
  c.n_grid = len > 0 ? (int)len : 0;
  c.grid_min = gmin;
  c.grid_delta = (gmin + gstep) - gmin;
  c.trig = dfmi_trig_k();
  std::vector<double> tab((size_t)(c.n_grid > 0 ? c.n_grid : 1) * ndata);
  std::vector<double> row(ndata + 2);
  for (int g = 0; g < c.n_grid; ++g) {
    dfmi_bessel_table(gmin + g * c.grid_delta, ndata, row.data());
    for (int i = 0; i < ndata; ++i) tab[(size_t)g * ndata + i] = row[i + 1];
  }
  for (long s = 0; s < n; ++s) {
    double p[4] = {guess[s * 4], guess[s * 4 + 1], guess[s * 4 + 2], guess[s * 4 + 3]};
    double ssq;
    if (force_general == 3) {  // the many-harmonic path (lm.h kWideNd), any ndata
      const dfmi::QCol qc{qi, (uint32_t)s, n, ndata};
      status_out[s] = dfmi::fit_segment_q<dfmi::kWideNd, dfmi::QCol>(qc, ndata, tab.data(), c, p, ssq);
    } else if (force_general == 4) {  // the same, one walk per trial (kWideNdF, wide_full)
      const dfmi::QCol qc{qi, (uint32_t)s, n, ndata};
      status_out[s] = dfmi::fit_segment_q<dfmi::kWideNdF, dfmi::QCol>(qc, ndata, tab.data(), c, p, ssq);
    } else if (force_general == 2 && ndata <= 12) {  // nested (one-lane) descent: must equal the flattened one
      const dfmi::QGlobal qg{qi + s, n, ndata};
      status_out[s] = dfmi::fit_segment_q<12, dfmi::QGlobal, false>(qg, ndata, tab.data(), c, p, ssq);
    } else if (force_general)
      status_out[s] = dfmi::fit_segment<0>(qi + s, n, ndata, tab.data(), c, p, ssq);
    else if (ndata == 10)  // the exact-ndata variant the device dispatches for ndata = 10
      status_out[s] = dfmi::fit_segment<dfmi::kExactNd | 10>(qi + s, n, ndata, tab.data(), c, p, ssq);
    else if (ndata <= 12)
      status_out[s] = dfmi::fit_segment<12>(qi + s, n, ndata, tab.data(), c, p, ssq);
    else if (ndata <= 16)
      status_out[s] = dfmi::fit_segment<16>(qi + s, n, ndata, tab.data(), c, p, ssq);
    else
      status_out[s] = dfmi::fit_segment<0>(qi + s, n, ndata, tab.data(), c, p, ssq);
    for (int i = 0; i < 4; ++i) p_out[s * 4 + i] = p[i];
    ssq_out[s] = ssq;
  }
  return 0;
}
}
