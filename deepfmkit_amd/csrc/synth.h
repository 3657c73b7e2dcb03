// synth.h — the asd-mode trial generator on the device (the input side of the
// batched efficiency trials), one lane per trial.
//
// Restates, in numpy's operation order (compiled without FMA contraction):
//   numpy.random.RandomState(seed) legacy stream: MT19937 init_genrand seeding,
//     the 624-word twist, next_double = (a>>5 * 2^26 + b>>6) / 2^53, the polar
//     legacy_gauss with its cached second value, normal = 0.0 + scale * gauss;
//   asd_noise_arrays (reference physics.py:532-613, white sources: amplitude, df;
//     seed 1 + trial_num * 4, sources drawn in the reference's order);
//   _run_simulation_physics (physics.py:615-722): g = waveform(omega_mod t + psi) / max|g|
//     (cos, or a waveform of waveforms.py: synth_g),
//     phi_mod = (2 pi / fs) * cumsum((df + n_df) * g), the exact-delay np.interp at
//     t - (tau_m + tau_dl) and t - tau_r, phase, (amp + n_amp) * (1 + vis cos(phase)).
// Every function rounds operation by operation (no FMA contraction, whatever the
// translation unit's flags). Bit-exact with numpy where the operations are IEEE
// (+ - * / sqrt, the RNG words); cos / sin / log are the device's (within an ulp of
// the host libm's), so records agree with the host generator to ~1e-15 relative,
// not bit for bit.
#pragma once
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define DFMI_SY_HD __host__ __device__ __forceinline__
#else
#define DFMI_SY_HD static inline
#endif

#include "../../include/dfmi.h"
#include "dfmi_math.h"

namespace dfmi {

constexpr int kMtN = 624;
constexpr int kMtM = 397;

// MT19937 output tempering of one state word
DFMI_SY_HD uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

// numpy mt19937_next_double from two consecutive tempered words
DFMI_SY_HD double mt_double(uint32_t wa, uint32_t wb) {
#pragma clang fp contract(off)
  const int32_t a = (int32_t)(wa >> 5), b = (int32_t)(wb >> 6);
  return (a * 67108864.0 + b) / 9007199254740992.0;
}

// One twist step of word i from its operands (i + 1 and i + M modulo the ring,
// already in the state the sequential twist would see)
DFMI_SY_HD uint32_t mt_twist_word(uint32_t ki, uint32_t ki1, uint32_t km) {
  const uint32_t y = (ki & 0x80000000u) | (ki1 & 0x7fffffffu);
  return km ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
}

// The polar method's candidate from four consecutive tempered words:
// x1, x2 in (-1, 1), r2 = x1^2 + x2^2; accepted iff 0 < r2 < 1.
DFMI_SY_HD bool polar_candidate(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, double* x1, double* x2,
                                double* r2) {
#pragma clang fp contract(off)
  *x1 = 2.0 * mt_double(w0, w1) - 1.0;
  *x2 = 2.0 * mt_double(w2, w3) - 1.0;
  *r2 = *x1 * *x1 + *x2 * *x2;
  return !(*r2 >= 1.0 || *r2 == 0.0);
}

// f = sqrt(-2 log(r2) / r2) of an accepted candidate (legacy_gauss returns f*x2,
// then the cached f*x1)
DFMI_SY_HD double polar_scale(double r2) {
#pragma clang fp contract(off)
  return sqrt(-2.0 * log(r2) / r2);
}

// One generator's state, its words at key(i) (the caller's layout: interleaved
// across lanes on the device, contiguous on the host).
template <typename Key>
struct Mt {
  Key key;
  int pos;
  bool has_gauss;
  double gauss;

  // numpy mt19937_seed (legacy RandomState(int) seeding)
  DFMI_SY_HD void seed(uint32_t s) {
    for (int i = 0; i < kMtN; ++i) {
      key(i) = s;
      s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
    }
    pos = kMtN;
    has_gauss = false;
    gauss = 0.0;
  }

  DFMI_SY_HD void twist() {
    int i = 0;
    for (; i < kMtN - kMtM; ++i) key(i) = mt_twist_word(key(i), key(i + 1), key(i + kMtM));
    for (; i < kMtN - 1; ++i) key(i) = mt_twist_word(key(i), key(i + 1), key(i + (kMtM - kMtN)));
    key(kMtN - 1) = mt_twist_word(key(kMtN - 1), key(0), key(kMtM - 1));
    pos = 0;
  }

  DFMI_SY_HD uint32_t next32() {
    if (pos == kMtN) twist();
    return mt_temper(key(pos++));
  }

  DFMI_SY_HD double next_double() { return mt_double(next32(), next32()); }

  // numpy legacy_gauss (polar method; the second value is kept for the next call)
  DFMI_SY_HD double next_gauss() {
#pragma clang fp contract(off)
    if (has_gauss) {
      const double t = gauss;
      has_gauss = false;
      gauss = 0.0;
      return t;
    }
    double x1, x2, r2;
    uint32_t w[4];
    do {
      for (int j = 0; j < 4; ++j) w[j] = next32();
    } while (!polar_candidate(w[0], w[1], w[2], w[3], &x1, &x2, &r2));
    const double f = polar_scale(r2);
    gauss = f * x1;
    has_gauss = true;
    return f * x2;
  }
};

// np.interp(x, t, f) on the uniform grid t_k = k / f_samp (numpy's arr_interp:
// left / right values, exact hits return f[j], slope form (f[j+1]-f[j])/(t[j+1]-t[j])).
template <typename Arr>
DFMI_SY_HD double interp_grid(double x, const Arr& f, int64_t n, double f_samp) {
#pragma clang fp contract(off)
  if (x != x) return x;
  if (x < 0.0) return f(0);
  const double tl = (double)(n - 1) / f_samp;
  if (x > tl) return f(n - 1);
  int64_t j = (int64_t)(x * f_samp);
  if (j > n - 1) j = n - 1;
  if (j < 0) j = 0;
  double tj = (double)j / f_samp;
  while (j > 0 && tj > x) tj = (double)(--j) / f_samp;
  while (j < n - 1 && (double)(j + 1) / f_samp <= x) tj = (double)(++j) / f_samp;
  if (j == n - 1) return f(n - 1);
  if (tj == x) return f(j);
  const double tn = (double)(j + 1) / f_samp;
  const double fj = f(j), fn = f(j + 1);
  const double slope = (fn - fj) / (tn - tj);
  double r = slope * (x - tj) + fj;
  if (r != r) {
    r = slope * (x - tn) + fn;
    if (r != r && fj == fn) r = fj;
  }
  return r;
}

// np.max's step (NaN propagates)
DFMI_SY_HD double synth_gmax_step(double m, double g) { return (g > m || g != g || m != m) ? (m != m ? m : g) : m; }

// g_t of sample k (before the max-normalisation): waveform_func(phase_axis,
// **waveform_kwargs), phase_axis = omega_mod t + psi (physics.py:661), for the default
// cos and the waveforms of waveforms.py, in numpy's / scipy.signal's operation order:
//  1 second_harmonic_distortion: cos(tp) + d_amp cos(2 tp + d_phase)
//  2 triangle_wave = sawtooth(tp, width): tmod = np.mod(tp, 2 pi); tmod < w 2 pi ?
//    tmod / (pi w) - 1 : (pi (w + 1) - tmod) / (pi (1 - w)); NaN for w outside [0, 1]
//  3 square_wave = square(tp, duty): tmod < w 2 pi ? 1 : -1; NaN for w outside [0, 1]
//  4 dfm_like_wave: y = cos(tp); y += a_n cos(n tp) per harmonic, in dict order
//  5 dfm_wave: cos(phi + m cos(tp))
// (2 and 3 use IEEE operations only: bit-exact with scipy; np.mod restated by dfmi_pymod.)
DFMI_SY_HD double synth_g(const dfmi_synth_trial& p, int64_t k, double f_samp) {
#pragma clang fp contract(off)
  const double pi = 3.141592653589793;
  const double tp = p.omega_mod * ((double)k / f_samp) + p.psi;
  switch (p.waveform) {
    case 1:
      return cos(tp) + p.d_amp * cos(2.0 * tp + p.d_phase);
    case 2:
    case 3: {
      const double w = p.d_amp;
      if (w > 1.0 || w < 0.0) return __builtin_nan("");
      const double tmod = dfmi_pymod(tp, 2.0 * pi);
      const bool first = tmod < w * 2.0 * pi;
      if (p.waveform == 3) return first ? 1.0 : -1.0;
      return first ? tmod / (pi * w) - 1.0 : (pi * (w + 1.0) - tmod) / (pi * (1.0 - w));
    }
    case 4: {
      double y = cos(tp);
      for (int i = 0; i < p.n_harm && i < 8; ++i) y += p.harm_amp[i] * cos(p.harm_n[i] * tp);
      return y;
    }
    case 5:
      return cos(p.d_phase + p.d_amp * cos(tp));
    default:
      return cos(tp);
  }
}

// df_noisy * g_normalised of sample k: the cumsum's summand
DFMI_SY_HD double synth_v(const dfmi_synth_trial& p, int64_t k, double f_samp, double gmax, double nz_df) {
#pragma clang fp contract(off)
  const double gn = gmax != 0.0 ? synth_g(p, k, f_samp) / gmax : 0.0;
  return (p.df + nz_df) * gn;
}

// The signal at sample k from phi_mod (the whole vector) and the amplitude noise
template <typename Arr>
DFMI_SY_HD double synth_signal(const dfmi_synth_trial& p, int64_t k, int64_t n, double f_samp, const Arr& phi,
                               double nz_amp) {
#pragma clang fp contract(off)
  const double t = (double)k / f_samp;
  const double dl = p.dynamic ? (p.arml_mod_amp * sin(p.w_arm * t + p.arml_mod_psi) + 0.0) + p.dl0 : p.dl0;
  const double tau_dl = dl / p.c_light;
  const double pm_meas = interp_grid(t - (p.tau_m + tau_dl), phi, n, f_samp);
  const double pm_ref = interp_grid(t - p.tau_r, phi, n, f_samp);
  const double phase = p.w0c * ((p.tau_m + tau_dl) - p.tau_r) + (pm_meas - pm_ref);
  const double amp = p.amp + nz_amp;
  return amp * (1.0 + p.vis * cos(phase));
}

// One trial, one lane (the host check's form; the device runs the same helpers with
// a wave per trial, synth.hip). nz_amp / nz_df / phi: the lane's scratch vectors (n values),
// out(k): the signal. Returns nothing; every value is written through the accessors.
template <typename Key, typename Vec, typename Out>
DFMI_SY_HD void synth_trial(const dfmi_synth_trial& p, int64_t n, double f_samp, Key key, Vec nz_amp, Vec nz_df,
                            Vec phi, Out out) {
#pragma clang fp contract(off)
  // asd_noise_arrays: one RandomState(seed), white sources in the reference's order
  Mt<Key> mt{key, 0, false, 0.0};
  mt.seed(p.seed);
  for (int64_t k = 0; k < n; ++k) nz_amp(k) = p.s_amp != 0.0 ? 0.0 + p.s_amp * mt.next_gauss() : 0.0;
  for (int64_t k = 0; k < n; ++k) nz_df(k) = p.s_df != 0.0 ? 0.0 + p.s_df * mt.next_gauss() : 0.0;
  // g_t normalised by max|g_t|
  double gmax = 0.0;
  for (int64_t k = 0; k < n; ++k) gmax = synth_gmax_step(gmax, fabs(synth_g(p, k, f_samp)));
  // phi_mod = (2 pi / fs) * cumsum(df_noisy * g_normalised)
  double acc = 0.0;
  for (int64_t k = 0; k < n; ++k) {
    const double v = synth_v(p, k, f_samp, gmax, nz_df(k));
    acc = k == 0 ? v : acc + v;
    phi(k) = p.cphi * acc;
  }
  for (int64_t k = 0; k < n; ++k) out(k) = synth_signal(p, k, n, f_samp, phi, nz_amp(k));
}

#if defined(__HIPCC__)
// synth.hip: scratch bytes for ntrial trials of n samples, and the launch.
size_t synth_scratch_bytes(int64_t ntrial, int64_t n);
hipError_t synth_launch(const dfmi_synth_trial* d_trials, int64_t ntrial, int64_t n, double f_samp, void* scratch,
                        double* out, hipStream_t st);
#endif

}  // namespace dfmi
