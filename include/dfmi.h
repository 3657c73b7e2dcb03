/* dfmi.h — C ABI of libdfmi.so, the MI355X (gfx950) DFMI per-segment NLS readout.
 *
 * Every entry point takes plain pointers and sizes; nothing here knows about
 * torch or numpy. A pointer argument is a HOST pointer when `mem` is
 * DFMI_MEM_HOST (the library stages it through device memory it owns and
 * returns after the results are back on the host) or a DEVICE pointer when
 * `mem` is DFMI_MEM_DEVICE (the library only enqueues kernels on `stream`, a
 * hipStream_t or NULL for the null stream, and returns without synchronising).
 * The library keeps no caller pointer after a call returns. HIP is initialised
 * lazily on the first call (never at load time), so the .so is safe to load in
 * a process that later forks (fitters.py:422 / experiments.py:381 Pools): a child
 * forked BEFORE the parent's first GPU call initialises HIP for itself. The library
 * records the pid of the process whose call first initialised HIP; a call from any
 * other pid — a child forked AFTER that point, which inherits HIP state it cannot
 * use — returns DFMI_ERR_HIP before touching the HIP runtime, and dfmi_last_error()
 * names both pids (fork first, or use the 'spawn' start method;
 * deepfmkit_amd/csrc/fork_guard.h).
 *
 * Return value: 0 on success, a negative DFMI_ERR_* code otherwise; the
 * message is in dfmi_last_error(). Numerical non-convergence is NOT an error:
 * it is the per-segment status 0/1/2 of fit.py:334-349, and a singular damped
 * system yields a zero step exactly as fit.py:197-204.
 *
 * Reference interfaces replaced (file:line in mdovale/DeepFMKit):
 *   dfmi_demod       calculate_quadratures (fit.py:18-66) + the per-buffer means of
 *                    fitters.py:45-49/380-384/436-440 and dc = mean(buffer)
 *                    (fitters.py:57/391/446)
 *   dfmi_lm          fit.fit (fit.py:322-361) incl. _run_lma_fit, msolve, coeffs,
 *                    ssqf, _find_best_initial_guess (fit.py:68-320), applied per
 *                    chunk with the warm start of _process_fit_chunk (fitters.py:13-60)
 *   dfmi_nls_record  StandardNLSFitter._fit_sequential / _fit_parallel
 *                    (fitters.py:370-428) for one or more records (channels)
 *   dfmi_ekf         EKFFitter.fit (fitters.py:214-320), pre-reductions by the caller
 *   dfmi_ekf_fit     EKFFitter.fit whole: np.mean / np.var on the device (fitters.py:253, 256)
 *   dfmi_record_moments  np.mean / np.var of records in numpy's summation order
 *   dfmi_synth_asd   SignalGenerator asd mode (physics.py:423-722, white noise) per
 *                    trial, the input side of workers.run_efficiency_trial batches
 *   dfmi_wdfmi_fit   WDFMI_NLSFitter / WDFMI_OrthogonalFitter / WDFMI_SequentialFitter /
 *                    HWDFMI_Fitter .fit (fitters.py:481-891)
 */
#ifndef DFMI_H
#define DFMI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DFMI_OK 0
#define DFMI_ERR_ARG (-1)
#define DFMI_ERR_HIP (-2)
#define DFMI_ERR_NODEV (-3)
#define DFMI_ERR_UNSUPPORTED (-4)

#define DFMI_MEM_HOST 0
#define DFMI_MEM_DEVICE 1

#define DFMI_MAX_LAMBDA 16

/* Numerical constants of fit.py:5-16 and the lambda ladder of fit.py:222.
 * The Python shim fills this from the live `deepfmkit_amd.fit` module globals
 * at call time (the reference's benchmark notebook overwrites them). */
typedef struct dfmi_lm_config {
  int32_t max_lma_steps;          /* MAX_LMA_STEPS (100) */
  int32_t n_lambda;               /* <= DFMI_MAX_LAMBDA */
  double lambdas[DFMI_MAX_LAMBDA];/* [0,1e-7,1e-5,1e-3,1e-1,1,10,100] */
  double min_step_norm;           /* 1e-15 (fit.py:230) */
  double conv_improve;            /* LMA_CONVERGENCE_IMPROVE (1e-9) */
  double conv_param_change;       /* LMA_CONVERGENCE_PARAM_CHANGE (1e-9) */
  double fitok_threshold;         /* FITOK_THRESHOLD (1e-3) */
  double m_grid_min;              /* M_GRID_MIN (5.0) */
  double m_grid_max;              /* M_GRID_MAX (30.0) */
  double m_grid_step;             /* M_GRID_STEP (0.5) */
  double bessel_amp_threshold;    /* BESSEL_AMP_THRESHOLD (0.05) */
  double sincos_amp_threshold;    /* SINCOS_AMP_THRESHOLD (0.1) */
} dfmi_lm_config;

/* Fill `cfg` with the reference defaults (fit.py:5-16, 222, 230). */
void dfmi_lm_config_default(dfmi_lm_config* cfg);

/* Demodulate nseg segments of R samples each.
 *   x[s*seg_stride + t], t < R           input samples (float64)
 *   qi[c*nseg + s], c < 2*ndata          output, component-major: c < ndata is
 *                                        Q_{c+1} = mean(x cos((c+1) w0 t)),
 *                                        c >= ndata is I_{c-ndata+1} (sin)
 *   dc[s]                                output, mean(x) of the segment
 * period: samples per basis period L (L*w0 = 2*pi*integer), 0 = detect from
 * w0, -1 = force the direct (per-sample sincos) kernel. */
int dfmi_demod(const double* x, int64_t nseg, int64_t seg_stride, int32_t R, int32_t ndata, double w0,
               int32_t period, double* qi, double* dc, int32_t mem, void* stream);

/* The record pipeline's demodulation layout ("rows"): one row of
 * dfmi_qi_row_stride(ndata) doubles per segment, rows[s*stride + pos]. Per block
 * of 8 harmonics b: 16 doubles [Q_{8b+1..8b+8} | I_{8b+1..8b+8}] (one 128-B line,
 * written by one store instruction; slots of harmonics > ndata are 0), and
 * dc = mean(segment) at pos dfmi_qi_row_dc(ndata). Same values as dfmi_demod
 * (bit-identical); only the layout differs. Needs 16-B aligned rows (x and
 * seg_stride even) and an even basis period 128 <= L <= 1024 (L = 200 at the
 * BASELINE configs); DFMI_ERR_UNSUPPORTED otherwise. */
int32_t dfmi_qi_row_stride(int32_t ndata);
int32_t dfmi_qi_row_dc(int32_t ndata);
int dfmi_demod_rows(const double* x, int64_t nseg, int64_t seg_stride, int32_t R, int32_t ndata, double w0,
                    int32_t period, double* rows, int32_t mem, void* stream);

/* Fit nseg demodulated segments.
 *   qi[c*nseg + s]                       input, layout of dfmi_demod
 *   guess_per_segment != 0: guess[s*4+i] seeds segment s (every segment its own chunk)
 *   guess_per_segment == 0: guess[0..3] seeds nchunk np.array_split chunks of the
 *                           nseg segments, warm start within a chunk
 *   params[i*nseg + s], i < 4            output amp, m, phi, psi (normalised)
 *   ssq[s], status[s]                    output */
int dfmi_lm(const double* qi, int64_t nseg, int32_t ndata, const double* guess, int32_t guess_per_segment,
            int64_t nchunk, const dfmi_lm_config* cfg, double* params, double* ssq, int32_t* status,
            int32_t mem, void* stream);

/* Whole StandardNLSFitter pass over nrec records (channels) of nbuf buffers.
 *   x[r*rec_stride + b*R + t]            input samples
 *   init_guess[r*4 + i]                  per-record default seed [init_a, init_m, 0, init_psi]
 *   parallel == 0: one warm-start chain over all nbuf buffers (fitters.py:370-393)
 *   parallel != 0: buffer 0 fitted from init_guess, then buffers 1..nbuf-1 split
 *                  into nchunk chunks seeded with buffer 0's result
 *                  (fitters.py:395-428; nchunk >= nbuf-1 = every buffer its own chunk)
 *   out[col*(nrec*nbuf) + r*nbuf + b]    col = 0 amp, 1 m, 2 phi, 3 psi, 4 dc, 5 ssq
 *   fitok[r*nbuf + b]                    status 0/1/2 */
int dfmi_nls_record(const double* x, int64_t nrec, int64_t rec_stride, int64_t nbuf, int32_t R, int32_t ndata,
                    double w0, int32_t period, const double* init_guess, int32_t parallel, int64_t nchunk,
                    const dfmi_lm_config* cfg, double* out, int32_t* fitok, int32_t mem, void* stream);

/* Per-sample EKF (fitters.py:214-320) over nrec independent channels, each a serial
 * chain over its samples: up to 16 x CUs channels one 16-lane DPP row per channel (4 per
 * wave; ekf_rot_kernel with sin / cos by rotation between anchors when R % 4 == 0, else
 * ekf_row_kernel), more channels one lane per channel (ekf_lane_rot_kernel / ekf_kernel);
 * dfmi_set_tuning "ekf_row" / "ekf_rot" select. Up to "ekf_pit" (1024) channels of at least
 * "ekf_pit_min" (4096) samples run parallel in time instead (ekf_pit.h): relinearization
 * passes of an associative linear Kalman scan over blocks, each ending in the true EKF per
 * block, until the output snapshots are within 1e-13 (relative to max(1, |x|)) of the
 * iteration's fixed point by the bound rho / (1 - rho) x their last move between passes, rho
 * the contraction measured per channel on the device; a channel that stops contracting (3
 * passes in a row with rho >= 1, or too slow to meet the bound within the cap) or reaches the
 * cap "ekf_pit_passes" (0 = by length: n / 1600 within [48, 256]) is re-run by the sequential kernel above; the same states to
 * rounding (~1e-13). The parallel form reads how many channels still pass after
 * "ekf_pit_first" (5) passes and then every "ekf_pit_every" (2): one stream
 * synchronisation each, so a DFMI_MEM_DEVICE call on this path returns with its stream
 * drained. The path depends on nrec and n_samp only (the sequential kernels run when the
 * parallel form's scratch cannot be allocated). x[r*rec_stride + k], k < n_samp. x0[r*5+i] initial state (dc included),
 * p0_diag[5], q_diag[5], r_val[r] measurement variance, w_m = 2*pi*f_mod,
 * f_samp; snapshots every R samples into states[(r*nbuf + b)*5 + i]. */
int dfmi_ekf(const double* x, int64_t nrec, int64_t rec_stride, int64_t n_samp, const double* x0,
             const double* p0_diag, const double* q_diag, const double* r_val, double w_m, double f_samp,
             int32_t R, int64_t nbuf, double* states, int32_t mem, void* stream);

/* EKFFitter.fit (fitters.py:214-320) whole: as dfmi_ekf, with the two whole-record
 * pre-reductions on the device, bit-exact with numpy: x0 = [init4[0..3],
 * np.mean(record)] (fitters.py:253) and the measurement variance r_val[0] for every
 * record, or np.var(record) when r_val is NULL (fitters.py:256). init4 (4 doubles:
 * init_a, init_m, init_phi, init_psi) and r_val live in `mem` like x. n_samp < 2^31. */
int dfmi_ekf_fit(const double* x, int64_t nrec, int64_t rec_stride, int64_t n_samp, const double* init4,
                 const double* p0_diag, const double* q_diag, const double* r_val, double w_m, double f_samp,
                 int32_t R, int64_t nbuf, double* states, int32_t mem, void* stream);

/* Passes the last dfmi_ekf / dfmi_ekf_fit call on this thread ran per channel (nrec as
 * that call's): 0 = sequential kernels, k > 0 = converged after k passes, -k = stopped
 * after k passes (not contracting, or the cap) and re-run by the sequential kernel. Copied
 * to the host by that call itself: no device access here; valid until the next EKF call on
 * this thread (a call that fails or takes the sequential path reports zeros). */
int dfmi_ekf_pit_passes(int32_t* passes, int64_t nrec);

/* Diagnostics of the stop rule: with dfmi_set_tuning("ekf_pit_trace", 1) during the last
 * EKF call on this thread (parallel form), moves[r*max_pass + p] = channel r's largest
 * relative move of its block-entry states in pass p (NaN for pass 0, whose previous entry
 * does not exist, and for passes not run). DFMI_ERR_ARG when that call kept no trace. */
int dfmi_ekf_pit_trace(double* moves, int64_t nrec, int32_t max_pass);

/* np.mean / np.var of nrec float64 records x[r*rec_stride .. + n] (1 <= n < 2^31),
 * bit-exact with numpy's pairwise summation (numpy 2.x _methods._mean / _var); var
 * may be NULL. One workgroup per record. */
int dfmi_record_moments(const double* x, int64_t nrec, int64_t rec_stride, int64_t n, double* mean, double* var,
                        int32_t mem, void* stream);

/* ---- Trial synthesis (input side of the batched efficiency trials) ----
 * One asd-mode channel per trial, as SignalGenerator.generate(mode='asd') makes it
 * (reference physics.py:423-473, white noise sources 532-613, exact-delay model
 * 615-722) for the default cosine waveform or one of the waveforms of waveforms.py:
 * numpy's legacy RandomState(seed) stream
 * (MT19937 + polar gauss) restated on the device. Every field is the reference's
 * scalar expression, evaluated by the caller with Python/numpy floats. */
typedef struct dfmi_synth_trial {
  uint32_t seed;        /* 1 + trial_num * 4 (asd_noise_arrays' RandomState) */
  int32_t dynamic;      /* 1: main channel (arm-length modulation term), 0: witness */
  double omega_mod;     /* 2 * np.pi * laser.f_mod */
  double psi;           /* laser.psi */
  double df;            /* laser.df */
  double cphi;          /* 2 * np.pi / fs, fs = 1 / (t[1] - t[0]) */
  double w_arm;         /* 2 * np.pi * ifo.arml_mod_f */
  double arml_mod_amp;  /* ifo.arml_mod_amp */
  double arml_mod_psi;  /* ifo.arml_mod_psi */
  double dl0;           /* ifo.phi * laser.wavelength / (2 * np.pi) */
  double c_light;       /* scipy.constants.c */
  double tau_m;         /* ifo.meas_arml / c */
  double tau_r;         /* ifo.ref_arml / c */
  double w0c;           /* 2 * np.pi * (c / laser.wavelength + 0.0) */
  double amp;           /* laser.amp */
  double vis;           /* laser.visibility */
  double s_amp;         /* laser.amp_n * np.sqrt(f_samp / 2.0), 0: no draws */
  double s_df;          /* laser.df_n * np.sqrt(f_samp / 2.0), 0: no draws */
  int32_t waveform;     /* g(tp), tp = omega_mod * t + psi (laser.waveform_func, waveforms.py):
                           0: cos(tp) (the default waveform);
                           1: second_harmonic_distortion (waveforms.py:4-23):
                              cos(tp) + d_amp * cos(2 * tp + d_phase);
                           2: triangle_wave = scipy.signal.sawtooth(tp, width = d_amp) (:25-31);
                           3: square_wave = scipy.signal.square(tp, duty = d_amp) (:33-43);
                           4: dfm_like_wave (:45-64): cos(tp) + sum_i harm_amp[i] * cos(harm_n[i] * tp);
                           5: dfm_wave (:66-90): cos(d_phase + d_amp * cos(tp)) */
  int32_t waveform_pad;
  double d_amp;         /* 1: distortion_amp; 2: width; 3: duty; 5: m */
  double d_phase;       /* 1: distortion_phase; 5: phi */
  int32_t n_harm;       /* 4: number of harmonics (<= 8), the harmonics dict in insertion order */
  int32_t harm_pad;
  double harm_n[8];     /* 4: harmonic numbers (the dict keys) */
  double harm_amp[8];   /* 4: their fractional amplitudes */
} dfmi_synth_trial;

/* out[r*n_samp + k] = trial r's signal sample k (t_k = k / f_samp), one lane per
 * trial. trials: host array; out in `mem`. Records agree with numpy's to ~1e-15
 * (the device's cos / sin / log), bit-exact elsewhere. */
int dfmi_synth_asd(const dfmi_synth_trial* trials, int64_t ntrial, int64_t n_samp, double f_samp, double* out,
                   int32_t mem, void* stream);

/* ---- Counter-based snr-mode input (bench / tests of sharded records) ----
 * The signal of SignalGenerator._generate_with_snr (physics.py:475-530, ideal signal
 * physics.py:493-518, is_dynamic=False) for samples [idx0, idx0 + n) of an unbounded
 * record: sample i = amp*(1 + visibility*cos(phi + m*cos(2*pi*f_mod*t + psi)))
 * + noise_std*z_i with t = (i mod period)/f_samp (period 0: t = i/f_samp) and z_i a
 * standard normal from Philox4x32-10 (key = seed, counter = (i>>1, stream, 0),
 * Box-Muller: z_2j = r*cos(2*pi*u2), z_2j+1 = r*sin(2*pi*u2)). Sample i depends only
 * on (params, i): any rank can regenerate any segment bit for bit at any world size.
 * Replaces the reference's RandomState(trial_num).randn stream, which cannot be split
 * (noise_std is the caller's physics.py:520-530 value). out[k] = sample idx0 + k. */
typedef struct dfmi_snr_params {
  uint64_t seed;
  uint32_t stream;     /* independent streams under one seed (e.g. channels) */
  int32_t period;      /* samples per modulation cycle (f_samp/f_mod when integer), or 0 */
  double f_samp, f_mod;
  double amp, visibility, m, phi, psi;
  double noise_std;
} dfmi_snr_params;

int dfmi_synth_snr(const dfmi_snr_params* prm, int64_t idx0, int64_t n, double* out, int32_t mem, void* stream);

/* Diagnostics (GPU parity of scipy.special.jv, fit.py:106-108, 160, 275-276): the
 * device Bessel code the fit kernels inline, on caller points.
 * out[i*(nmax+1) + k] = J_k(x[i]), k <= nmax. method 0: the general path's two-pass
 * Miller walk (any nmax); 1: the register path of ndata <= 12 (nmax <= 13);
 * 2: the register path of ndata <= 16 (nmax <= 17). */
int dfmi_bessel_eval(const double* x, int64_t nx, int32_t nmax, int32_t method, double* out, int32_t mem,
                     void* stream);

/* ---- Witness-based fitters (EXPERIMENTAL in the reference) ----
 * Replace, per record (main channel + witness channel):
 *   DFMI_WDFMI_NLS    WDFMI_NLSFitter.fit        fitters.py:481-570 (least_squares(method='lm'))
 *   DFMI_WDFMI_ORTHO  WDFMI_OrthogonalFitter.fit fitters.py:572-648 (Nelder-Mead + VarPro)
 *   DFMI_WDFMI_SEQ    WDFMI_SequentialFitter.fit fitters.py:650-776 (Brent, bounded Brent, lstsq)
 *   DFMI_HWDFMI       HWDFMI_Fitter.fit          fitters.py:778-891 (Brent + VarPro)
 * with the witness template of _get_phase_modulation_basis (fitters.py:88-122) or
 * _get_total_laser_phase (fitters.py:124-162) built from the witness's first R samples. */
#define DFMI_WDFMI_NLS 0
#define DFMI_WDFMI_ORTHO 1
#define DFMI_WDFMI_SEQ 2
#define DFMI_HWDFMI 3

typedef struct dfmi_wdfmi_config {
  int32_t method;     /* DFMI_WDFMI_* / DFMI_HWDFMI */
  int32_t ndata;      /* WDFMI_NLS harmonics (10), <= 32 */
  int32_t ndata_psi;  /* WDFMI_SEQ stage-2 harmonics (40), <= 64 */
  int32_t period;     /* basis period of the harmonic sums: 0 detect, -1 per-sample sincos */
  double f_samp;      /* main_raw.f_samp */
  double f_mod;       /* laser_cfg.f_mod */
  double df;          /* laser_cfg.df (W-DFMI template scale, m = 2 pi df tau) */
  double f_ref;       /* HW-DFMI reference frequency (witness ifo.arml_mod_f) */
  double tau_init;    /* first guess of tau: the caller applies the reference's rule per
                         method (delta_l / c, 0 when df <= 0 for ortho/seq, init_tau for HW) */
  double init_a, init_phi, init_psi;
} dfmi_wdfmi_config;

/* Fit nrec records of nbuf buffers of R samples.
 *   x[r*rec_stride + b*R + k]            main channel samples
 *   witness[r*wit_stride + k], k < R     witness channel (wit_stride 0: one witness for all)
 *   out[col*(nrec*nbuf) + r*nbuf + b]    col = 0 amp, 1 m, 2 phi, 3 psi, 4 tau, 5 dc, 6 ssq
 *   fitok[r*nbuf + b]                    the reference's fitok column
 * NLS / ORTHO / HW warm-start buffer b from buffer b-1 (one workgroup per record);
 * SEQ fits every buffer independently. R <= 16384. A rank-deficient VarPro system
 * costs +inf (the reference's ORTHO raises IndexError there). */
int dfmi_wdfmi_fit(const double* x, int64_t nrec, int64_t rec_stride, int64_t nbuf, int32_t R,
                   const double* witness, int64_t wit_stride, const dfmi_wdfmi_config* cfg, double* out,
                   int32_t* fitok, int32_t mem, void* stream);

/* Performance tuning hook, process-wide; each call works on a snapshot taken at its
 * start. Results are unaffected (ekf_rot, ekf_pit*: rounding only). Keys: "demod_kernel" (1 phase bins in LDS where they
 * apply [default], 0 cycle-aligned fold), "lm_general" (1 = two-pass general LM path
 * for every ndata), "demod_spw" (segments per wave the bin grid is sized for; 0 =
 * persistent), "demod_wide" (1 [default]: component-major QI through the many-harmonic
 * kernel demod_wide_kernel from "demod_wide_from" (13) harmonics or below "demod_wide_rmax"
 * (2000) samples per segment — the record pipeline then leaves its fused row layout; 0: the
 * bin / fold kernels; 2: demod_wide_kernel wherever its geometry applies; QI within ~1e-14
 * relative of the bin kernel's), "demod_wide_k" (segments per wave, 0 = 8; 2 / 4 / 8),
 * "demod_wide_half" (1 [default]: half-wave contraction at 2 ndata + 1 <= 32; same bits),
 * "demod_wide_dbg" (diagnostics: bit 0 no contraction, bit 1 no stores, bit 2 segment-by-segment
 * fold — results invalid with bits 0 / 1), "ekf_row" (EKF row kernel up to ekf_row x 16 x CUs channels, 0 = lane
 * kernel only), "ekf_rot" (1 [default]: the row kernel takes sin / cos by rotation between
 * anchors of 16 (8, 4) samples where R % 4 == 0, ekf_rot_kernel; rounding only),
 * "wdfmi_accel" (bit 0: W-DFMI time axis without division, bit 1: template slopes in
 * LDS; both exact), "lm_ladder" (LM launches of at most lm_ladder x CUs
 * chains or segments run the parallel lambda ladder, 8 lanes per item: warm-start chains,
 * small batches; 0 = never; default 32; same bits), "ws_streams" (caller streams whose
 * scratch workspaces are kept per device, default 4: a DFMI_MEM_DEVICE call from a stream
 * beyond that many first DRAINS THE DEVICE (hipDeviceSynchronize) and frees the least
 * recently used stream's workspaces — a caller cycling over more streams serialises every
 * call, and such a call must not be made while a stream is being captured into a graph;
 * raise the key to the number of streams in use), "ekf_pit" (EKF parallel in time for up
 * to this many channels, default 1024; 0 = the sequential kernels always), "ekf_pit_min"
 * (samples per channel below which the sequential kernels run, default 4096),
 * "ekf_pit_block" (samples per block, 0 = ~n nrec^(2/3) / 16384, at least 16), "ekf_pit_passes"
 * (pass cap before the sequential kernel, default 0 = n / 1600 within [48, 256]), "ekf_pit_first" / "ekf_pit_every"
 * (passes before the first / between later host reads of the channels still passing, 5 / 2),
 * "ekf_pit_tol" (the stop rule's bound 10^-k, default 13), "ekf_pit_stall" (non-contracting
 * passes in a row before the sequential kernel, default 3), "ekf_pit_measure" (0 [default]:
 * the rule's move is the output snapshots'; 1, diagnostics: the block-entry states'), "ekf_pit_trace" (0 / 1,
 * dfmi_ekf_pit_trace), "ekf_pit_seq" (1 [default]; 0, diagnostics only: an unconverged
 * channel keeps its last pass's states instead of the sequential kernel's), "ekf_pit_head"
 * (samples the sequential EKF seeds the trajectory with, default 256), "ekf_pit_fused" (1
 * [default]: the EKF and the next pass's fold in one kernel per pass; 0: separate kernels),
 * "ekf_pit_topfix" (1 [default]: a scan top level of at most 4 elements is folded by the
 * fix-up below it instead of its own launch; rounding only), "ekf_pit_slow_from" (pass from
 * which the rule's "too slow to meet the bound within the
 * cap" extrapolation counts, default 16), "ekf_pit_overlap" (where the sequential re-runs of
 * handed-over channels go: 0 [default] one launch after the passes on the caller's stream; 3 /
 * 2 / 1 at each host check on a pool of three / one high- / one default-priority stream beside
 * the passes — measured slower; same states), "lm_wide" (1 [default]: beyond 16 harmonics the
 * many-harmonic LM, closed-form sums over a lean Miller walk; 0: the literal general path;
 * rounding only), "lm_wide_lds" (the largest ndata whose QI the many-harmonic LM stages in LDS
 * per lane, default 20; same bits), "lm_wide_fused" (1 [default]: one walk per trial for ssqf
 * and coeffs beyond lm_wide_lds, in the ladder and in the seed; same bits), "lm_split" /
 * "lm_split_from" (0 [default] / 41: P = 2 or 4 lanes per segment from that ndata — measured
 * slower; rounding only), "seed_wave_split" (1 [default]: the seed beyond 16 harmonics fitted by
 * the whole wave as 8 lambda rungs x 8 harmonic shares; 0: 8-lane groups each running the
 * whole fit; rounding only), "lm_ladder_split" (the ladder beyond 16 harmonics for at most this
 * many items per CU, default 4: one wave per item as 8 rungs x 8 harmonic shares; 0 = 8 lanes
 * per item; rounding only),
 * "probe" (1 =
 * diagnostics timestamp buffer on the current device, dfmi_probe_read). */
int dfmi_set_tuning(const char* key, int64_t value);

/* Current value of a tuning key (see dfmi_set_tuning). */
int dfmi_get_tuning(const char* key, int64_t* value);

/* Measurement hook: with enable != 0, dfmi_nls_record records timing events on its
 * stream around the fused seed + demodulation launch and the LM launch of the record
 * pipeline (current device). dfmi_step_timing_read waits for them and returns the
 * summed kernel-span times (ms) of the steps recorded since the last read (at most 65,536
 * steps wait to be read; later calls are not marked, *nsteps says how many were). A call
 * that fails part-way records no step. */
int dfmi_step_timing(int32_t enable);
int dfmi_step_timing_read(double* demod_ms, double* lm_ms, int64_t* nsteps);

/* Frees every scratch workspace of the current device after waiting for it to drain
 * (workspaces are kept per caller stream, at most "ws_streams" streams [default 4], least
 * recently used freed first). */
int dfmi_release_workspaces(void);

/* Diagnostics: with dfmi_set_tuning("probe", 1) some kernels record
 * s_memrealtime (100 MHz) timestamps; copies the first n (<= 16) of them
 * (synchronises the device). [0..2] seed entry / after fold / after fit,
 * [3] bin demod workgroup 0 entry, [4] last workgroup entry, [5] workgroup 0 exit. */
int dfmi_probe_read(int64_t* out, int32_t n);

/* Period (samples) the fold kernel would use for this w0, R, ndata; 0 if none. */
int32_t dfmi_detect_period(double w0, int32_t R, int32_t ndata);

/* ---- The reference's text formats (host code, no GPU) ----
 * raw_data / fit_data: 13 header lines ('%'-prefixed; lines 3..11 carry the numbers
 * parse_header extracts by keeping only the characters "0123456789."), then one
 * row per sample (raw: one column per channel, read with pandas sep=' ') or per
 * segment (fit: ssq amp m phi psi dc per channel, read with numpy.genfromtxt).
 * Replaces core.py:129-174 (parse_header), 259-286 (load_raw), 288-332 (load_fit)
 * and data.py:178-208 (DeepFitObject.to_txt). Errors: negative return and
 * dfmi_txt_last_error(). */
#define DFMI_TXT_RAW 0
#define DFMI_TXT_FIT 1
#define DFMI_TXT_SINGLE_SPACE 0 /* pandas.read_csv(sep=' '): every space separates */
#define DFMI_TXT_WHITESPACE 1   /* numpy.genfromtxt: blank runs separate, '#' comments,
                                   rows whose field count differs from the first are skipped */
typedef struct dfmi_txt_header {
  int32_t kind;      /* DFMI_TXT_RAW | DFMI_TXT_FIT */
  int32_t channels;  /* line 3 */
  int64_t t0;        /* line 4 */
  double f_samp;     /* line 5 */
  double f_mod;      /* line 6 */
  int32_t n;         /* fit: line 7 */
  int32_t R;         /* fit: line 8 */
  double fs;         /* fit: line 9 */
} dfmi_txt_header;

int dfmi_txt_parse_header(const char* path, int32_t kind, dfmi_txt_header* hdr);
/* Data rows after `skip` lines and the largest field count of a row. */
int dfmi_txt_shape(const char* path, int32_t skip, int32_t mode, int64_t* rows, int32_t* cols);
/* out[k*rows + i] = column cols[k] of data row i (NaN when missing/invalid);
 * `threads` host threads parse disjoint line ranges. */
int dfmi_txt_read(const char* path, int32_t skip, int32_t mode, int32_t ncol, const int32_t* cols, double* out,
                  int64_t rows, int32_t threads);
/* `header` verbatim, then n rows "ssq amp m phi psi dc \n" with every value in
 * CPython repr() digits (data.py:198-207 writes str(float)). */
int dfmi_fit_txt_write(const char* path, const char* header, const double* ssq, const double* amp, const double* m,
                       const double* phi, const double* psi, const double* dc, int64_t n);
/* CPython repr(v) into buf; returns its length or a negative error. */
int dfmi_py_repr(double v, char* buf, int32_t cap);
const char* dfmi_txt_last_error(void);

/* Number of visible HIP devices (initialises HIP). */
int dfmi_device_count(void);

/* Message of the last failed call on this thread ("" if none). */
const char* dfmi_last_error(void);

/* Library/ABI version, e.g. "dfmi 0.3 gfx950". */
const char* dfmi_version(void);

/* Kernel variant of the last demodulation (or EKF fit) this THREAD launched, with the
 * template arguments of the instance (loads in flight and prefetched chunks come from the
 * build), e.g. "demod_seed_bins_kernel<2,12,4,10> (prefetch 4)" (the record pipeline's
 * fused seed + demodulation), "demod_bins_kernel<2,10,rows,4> (prefetch 4)" (dfmi_demod_rows),
 * "ekf_rot_kernel", "ekf_row_kernel", "ekf_lane_rot_kernel", "ekf_kernel" ("" before the
 * first one). Diagnostics/profiling. */
const char* dfmi_last_demod_kernel(void);

#ifdef __cplusplus
}
#endif

#endif /* DFMI_H */
