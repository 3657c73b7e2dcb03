"""Simulation configuration objects and the synthetic-input generator.

Only what the NLS readout path needs as INPUT is restated here (SURVEY.md §8a row
a16): the configuration containers and the snr-mode generator of
physics.py:475-530, plus the zero/white-noise subset of the asd mode used by
workers.run_single_trial (physics.py:423-473, 615-722).  Coloured (1/f^alpha)
noise needs `pyplnoise`, which is absent from this image: requesting it raises.

The snr-mode restatement keeps the reference's numpy operation order, so for a
given seed the generated record is bit-identical to the reference's (pinned by
the SHA-256 values in tests/golden/manifest.json).
"""
from __future__ import annotations

import logging
from typing import Any, Callable, Dict, Optional

import numpy as np
import scipy.constants as sc

from .data import DeepRawObject

log = logging.getLogger(__name__)


def cosine_waveform(t_phase):
    """The default frequency-modulation waveform (reference physics.py:15-51)."""
    return np.cos(t_phase)


class LaserConfig:
    """Laser source parameters (reference physics.py:15-51)."""

    def __init__(self, label="laser_source", psi=None):
        self.label = label
        self.wavelength = 1.064e-6
        self.amp = 1.0
        self.visibility = 1.0
        self.f_mod = 1000
        self.df = 3e9
        self.psi = psi if psi else 0.0
        self.waveform_func: Callable[..., np.ndarray] = cosine_waveform
        self.waveform_kwargs: Dict[str, Any] = {}
        self.f_n = 0.0
        self.df_n = 0.0
        self.amp_n = 0.0


class InterferometerConfig:
    """Optical path parameters (reference physics.py:213-237)."""

    def __init__(self, label="interferometer_path"):
        self.label = label
        self.phi = 0.0
        self.ref_arml = 0.1
        self.meas_arml = 0.3
        self.arml_mod_f = 5.0
        self.arml_mod_amp = 0.0
        self.arml_mod_psi = 0.0
        self.arml_mod_n = 0.0


class DFMIObject:
    """One simulation channel = laser + interferometer (reference physics.py:239-296)."""

    def __init__(self, label, laser_config, ifo_config, f_samp=200000):
        self.label = label
        self.laser = laser_config
        self.ifo = ifo_config
        self.f_samp = float(f_samp)
        self.N = 0
        self.simtime = None
        self.fit_n = 20
        self.f_fit = float(self.laser.f_mod / self.fit_n)

    @property
    def m(self):
        delta_l = self.ifo.meas_arml - self.ifo.ref_arml
        if delta_l == 0:
            return 0.0
        return 2 * np.pi * self.laser.df * delta_l / sc.c


def set_laser_df_for_effect(laser: LaserConfig, ifo: InterferometerConfig, m):
    """helpers.py:10-14: choose laser.df so that the channel's m equals `m`."""
    opd = np.abs(ifo.meas_arml - ifo.ref_arml)
    laser.df = (m * sc.c) / (2 * sc.pi * opd)


class SignalGenerator:
    """Synthetic DFMI time series (reference physics.py:362-530)."""

    def generate(self, main_config, n_seconds, mode="asd", trial_num=0, witness_config=None, snr_db=None,
                 external_noise: Optional[dict] = None):
        if mode == "asd":
            return self._generate_with_asd(main_config, n_seconds, trial_num, witness_config, external_noise)
        if mode == "snr":
            if snr_db is None:
                log.error("SNR mode requires a value for 'snr_db'.")
                return {}
            return self._generate_with_snr(main_config, n_seconds, trial_num, snr_db)
        log.error(f"Unknown simulation mode: '{mode}'")
        return {}

    # --- snr mode: physics.py:475-530 ---------------------------------------
    def _generate_with_snr(self, cfg, n_seconds, trial_num, snr_db):
        num_samples = int(n_seconds * cfg.f_samp)
        t = np.arange(num_samples) / cfg.f_samp
        cfg.N = len(t)
        y = ideal_signal(cfg, t)
        y = add_white_noise(y, snr_db, trial_num)
        raw = DeepRawObject(data=y)
        raw.label = cfg.label
        raw.f_samp = cfg.f_samp
        raw.f_mod = cfg.laser.f_mod
        raw.t0 = 0
        raw.sim = cfg
        return {"main": raw}

    # --- asd mode, zero/white-noise subset: physics.py:423-473, 532-722 ------
    def _generate_with_asd(self, cfg, n_seconds, trial_num, witness_config, external_noise=None):
        num_samples = int(n_seconds * cfg.f_samp)
        t = np.arange(num_samples) / cfg.f_samp
        cfg.N = len(t)
        if external_noise:
            noise = {k: external_noise.get(k, 0.0) for k in ("laser_frequency", "amplitude", "df", "armlength")}
        else:
            noise = asd_noise_arrays(cfg, len(t), trial_num)
        out = {}
        for key, c, dyn in (("main", cfg, True), ("witness", witness_config, False)):
            if c is None:
                continue
            sig, phase, truth = exact_model_signal(c, t, noise, dyn)
            raw = DeepRawObject(data=sig)
            raw.label = c.label
            raw.f_samp = c.f_samp
            raw.f_mod = c.laser.f_mod
            raw.sim = c
            raw.phi = phase
            raw.phi_sim = truth
            out[key] = raw
        return out


def ideal_signal(cfg, t):
    """physics.py:493-518 with is_dynamic=False: A(1 + C cos(phi + m cos(w t + psi)))."""
    laser, ifo = cfg.laser, cfg.ifo
    omega_mod = 2 * np.pi * laser.f_mod
    phitot = ifo.phi + cfg.m * np.cos(omega_mod * t + laser.psi)
    return laser.amp * (1 + laser.visibility * np.cos(phitot))


def add_white_noise(clean, snr_db, trial_num):
    """physics.py:520-530: white Gaussian noise from RandomState(trial_num)."""
    ac = clean - np.mean(clean)
    power = np.mean(ac ** 2)
    std = np.sqrt(power / 10 ** (snr_db / 10.0))
    rng = np.random.RandomState(seed=trial_num)
    return clean + rng.randn(len(clean)) * std


def asd_noise_arrays(cfg, n_samples, trial_num=0):
    """physics.py:532-613, white/zero sources only (coloured needs pyplnoise)."""
    fs = cfg.f_samp
    params = [("laser_frequency", cfg.laser.f_n, 2.0), ("amplitude", cfg.laser.amp_n, 0.0),
              ("df", cfg.laser.df_n, 0.0), ("armlength", cfg.ifo.arml_mod_n, 2.0)]
    rng = np.random.RandomState(seed=1 + trial_num * len(params))
    out = {}
    for name, asd, alpha in params:
        if asd == 0.0:
            out[name] = 0.0
        elif name in ("amplitude", "df"):
            out[name] = rng.normal(scale=asd * np.sqrt(fs / 2.0), size=int(n_samples))
        else:
            raise NotImplementedError(
                f"coloured '{name}' noise (alpha={alpha}) needs pyplnoise, which is not installed")
    return out


def exact_model_signal(cfg, t, noise, is_dynamic):
    """physics.py:615-722: exact-delay model via the integrated FM waveform."""
    laser, ifo = cfg.laser, cfg.ifo
    omega_mod = 2 * np.pi * laser.f_mod
    g = laser.waveform_func(omega_mod * t + laser.psi, **laser.waveform_kwargs)
    gmax = np.max(np.abs(g))
    g = g / gmax if gmax != 0 else np.zeros_like(g)
    df_noisy = laser.df + noise.get("df", 0.0)
    dt = t[1] - t[0]
    fs = 1 / dt
    phi_mod = (2 * np.pi / fs) * np.cumsum(df_noisy * g)
    tau_r = ifo.ref_arml / sc.c
    tau_m = ifo.meas_arml / sc.c
    if not is_dynamic:
        dl = ifo.phi * laser.wavelength / (2 * np.pi)
    else:
        dl = (ifo.arml_mod_amp * np.sin(2 * np.pi * ifo.arml_mod_f * t + ifo.arml_mod_psi)
              + noise.get("armlength", 0.0) + ifo.phi * laser.wavelength / (2 * np.pi))
    tau_dl = dl / sc.c
    pm_meas = np.interp(t - (tau_m + tau_dl), t, phi_mod)
    pm_ref = np.interp(t - tau_r, t, phi_mod)
    f0 = (sc.c / laser.wavelength) + noise.get("laser_frequency", 0.0)
    phase = 2 * np.pi * f0 * ((tau_m + tau_dl) - tau_r) + (pm_meas - pm_ref)
    amp = laser.amp + noise.get("amplitude", 0.0)
    sig = amp * (1 + laser.visibility * np.cos(phase))
    truth = (2 * np.pi * sc.c / laser.wavelength) * ((tau_m + tau_dl) - tau_r)
    if np.isscalar(truth):
        truth = np.full_like(t, truth, dtype=float)
    return sig, phase, truth


# --- asd-mode trials on the device (dfmi_synth_asd) ---------------------------

SYNTH_MAX_HARM = 8  # dfm_like_wave harmonics dfmi_synth_asd evaluates
SYNTH_TRIAL_DTYPE = np.dtype([("seed", "<u4"), ("dynamic", "<i4")] + [(k, "<f8") for k in (
    "omega_mod", "psi", "df", "cphi", "w_arm", "arml_mod_amp", "arml_mod_psi", "dl0", "c_light", "tau_m", "tau_r",
    "w0c", "amp", "vis", "s_amp", "s_df")] + [("waveform", "<i4"), ("waveform_pad", "<i4"), ("d_amp", "<f8"),
                                                 ("d_phase", "<f8"), ("n_harm", "<i4"), ("harm_pad", "<i4"),
                                                 ("harm_n", "<f8", (SYNTH_MAX_HARM,)),
                                                 ("harm_amp", "<f8", (SYNTH_MAX_HARM,))])  # dfmi_synth_trial


def _real_scalar(v):
    return isinstance(v, (int, float, np.integer, np.floating)) and not isinstance(v, bool)


def _device_waveform(laser):
    """(code, d_amp, d_phase, harmonics) of a waveform dfmi_synth_asd evaluates
    (include/dfmi.h dfmi_synth_trial.waveform), or None: the default cosine and the
    waveforms of waveforms.py (reference waveforms.py:4-90) with scalar arguments."""
    from . import waveforms as W
    kw = dict(laser.waveform_kwargs or {})
    f = laser.waveform_func
    if not all(_real_scalar(v) or (k == "harmonics" and (v is None or isinstance(v, dict))) for k, v in kw.items()):
        return None
    if f is cosine_waveform and not kw:
        return 0, 0.0, 0.0, ()
    if f is W.second_harmonic_distortion and set(kw) <= {"distortion_amp", "distortion_phase"}:
        return 1, float(kw.get("distortion_amp", 0.0)), float(kw.get("distortion_phase", 0.0)), ()
    if f is W.triangle_wave and set(kw) <= {"width"}:
        return 2, float(kw.get("width", 0.5)), 0.0, ()
    if f is W.square_wave and set(kw) <= {"duty"}:
        return 3, float(kw.get("duty", 0.5)), 0.0, ()
    if f is W.dfm_like_wave and set(kw) <= {"harmonics"}:
        h = kw.get("harmonics")
        h = {2: 0.1, 3: 0.05} if h is None else h  # waveforms.py:58-59
        if len(h) > SYNTH_MAX_HARM or not all(_real_scalar(n) and _real_scalar(a) for n, a in h.items()):
            return None
        return 4, 0.0, 0.0, tuple((float(n), float(a)) for n, a in h.items())
    if f is W.dfm_wave and set(kw) <= {"m", "phi"}:
        return 5, float(kw.get("m", 1.0)), float(kw.get("phi", 0.0)), ()
    return None


def _put_waveform(rec, wf):
    rec["waveform"], rec["d_amp"], rec["d_phase"] = wf[0], wf[1], wf[2]
    rec["n_harm"] = len(wf[3])
    for i, (n, a) in enumerate(wf[3]):
        rec["harm_n"][i] = n
        rec["harm_amp"][i] = a


def device_synth_supported(cfg) -> bool:
    """dfmi_synth_asd covers the default cosine waveform and the waveforms of
    waveforms.py (second-harmonic distortion, triangle, square, dfm-like, dfm) with
    scalar arguments, white (or zero) amplitude / df noise and no frequency /
    arm-length noise sources."""
    laser, ifo = cfg.laser, cfg.ifo
    return _device_waveform(laser) is not None and laser.f_n == 0.0 and ifo.arml_mod_n == 0.0


def synth_trial_fields(cfg, trial_num, dynamic=True):
    """One dfmi_synth_trial: the scalar sub-expressions of asd_noise_arrays and
    exact_model_signal, evaluated here exactly as those numpy expressions do."""
    laser, ifo = cfg.laser, cfg.ifo
    seed = 1 + int(trial_num) * 4
    if not 0 <= seed <= 2 ** 32 - 1:
        raise ValueError("Seed must be between 0 and 2**32 - 1")
    fs_cfg = cfg.f_samp
    t01 = np.arange(2) / cfg.f_samp
    dt = t01[1] - t01[0]
    fs = 1 / dt
    f0 = (sc.c / laser.wavelength) + 0.0
    rec = np.zeros((), dtype=SYNTH_TRIAL_DTYPE)
    rec["seed"], rec["dynamic"] = seed, 1 if dynamic else 0
    rec["omega_mod"] = 2 * np.pi * laser.f_mod
    rec["psi"] = laser.psi
    rec["df"] = laser.df
    rec["cphi"] = 2 * np.pi / fs
    rec["w_arm"] = 2 * np.pi * ifo.arml_mod_f
    rec["arml_mod_amp"] = ifo.arml_mod_amp
    rec["arml_mod_psi"] = ifo.arml_mod_psi
    rec["dl0"] = ifo.phi * laser.wavelength / (2 * np.pi)
    rec["c_light"] = sc.c
    rec["tau_m"] = ifo.meas_arml / sc.c
    rec["tau_r"] = ifo.ref_arml / sc.c
    rec["w0c"] = 2 * np.pi * f0
    rec["amp"] = laser.amp
    rec["vis"] = laser.visibility
    rec["s_amp"] = laser.amp_n * np.sqrt(fs_cfg / 2.0) if laser.amp_n != 0.0 else 0.0
    rec["s_df"] = laser.df_n * np.sqrt(fs_cfg / 2.0) if laser.df_n != 0.0 else 0.0
    wf = _device_waveform(laser)
    if wf is None:
        raise ValueError("dfmi_synth_asd does not evaluate this waveform")
    _put_waveform(rec, wf)
    return rec


def synth_trial_table(cfgs, trial_nums, dynamic=True):
    """dfmi_synth_trial rows for many (cfg, trial_num): synth_trial_fields' expressions
    evaluated elementwise over the trials (numpy's vector ops round exactly as its scalar
    ones: the same bits as the per-trial form, tests/test_host_numerics.py)."""
    n = len(cfgs)
    if any(not device_synth_supported(c) for c in cfgs):
        bad = [i for i, c in enumerate(cfgs) if not device_synth_supported(c)]
        raise ValueError(f"trials {bad[:5]} need the host generator (custom waveform or coloured noise)")
    f_samp = float(cfgs[0].f_samp)
    if any(float(c.f_samp) != f_samp for c in cfgs):
        raise ValueError("synthesize_asd_trials: trials must share f_samp")
    seeds = 1 + np.asarray(trial_nums, dtype=np.int64) * 4
    if seeds.size and (seeds.min() < 0 or seeds.max() > 2 ** 32 - 1):
        raise ValueError("Seed must be between 0 and 2**32 - 1")

    def col(get):
        return np.fromiter((get(c) for c in cfgs), dtype=np.float64, count=n)

    f_mod, psi, df = col(lambda c: c.laser.f_mod), col(lambda c: c.laser.psi), col(lambda c: c.laser.df)
    wl, amp, vis = col(lambda c: c.laser.wavelength), col(lambda c: c.laser.amp), col(lambda c: c.laser.visibility)
    amp_n, df_n = col(lambda c: c.laser.amp_n), col(lambda c: c.laser.df_n)
    arm_f, arm_a, arm_p = (col(lambda c: c.ifo.arml_mod_f), col(lambda c: c.ifo.arml_mod_amp),
                           col(lambda c: c.ifo.arml_mod_psi))
    phi, meas, ref = col(lambda c: c.ifo.phi), col(lambda c: c.ifo.meas_arml), col(lambda c: c.ifo.ref_arml)
    wf = [_device_waveform(c.laser) for c in cfgs]
    t01 = np.arange(2) / f_samp
    fs = 1 / (t01[1] - t01[0])
    tab = np.zeros(n, dtype=SYNTH_TRIAL_DTYPE)
    tab["seed"], tab["dynamic"] = seeds.astype(np.uint32), 1 if dynamic else 0
    tab["omega_mod"] = 2 * np.pi * f_mod
    tab["psi"] = psi
    tab["df"] = df
    tab["cphi"] = 2 * np.pi / fs
    tab["w_arm"] = 2 * np.pi * arm_f
    tab["arml_mod_amp"] = arm_a
    tab["arml_mod_psi"] = arm_p
    tab["dl0"] = phi * wl / (2 * np.pi)
    tab["c_light"] = sc.c
    tab["tau_m"] = meas / sc.c
    tab["tau_r"] = ref / sc.c
    tab["w0c"] = 2 * np.pi * ((sc.c / wl) + 0.0)
    tab["amp"] = amp
    tab["vis"] = vis
    tab["s_amp"] = np.where(amp_n != 0.0, amp_n * np.sqrt(f_samp / 2.0), 0.0)
    tab["s_df"] = np.where(df_n != 0.0, df_n * np.sqrt(f_samp / 2.0), 0.0)
    for i, w in enumerate(wf):
        _put_waveform(tab[i], w)
    return tab


def synthesize_asd_trials(cfgs, trial_nums, n_seconds, dynamic=True):
    """The main channel (dynamic=True) or a witness channel (dynamic=False) of
    SignalGenerator.generate(cfg, n_seconds, mode='asd', trial_num=t) for every (cfg, t),
    generated on the GPU (dfmi_synth_asd) into one (ntrial, N) CUDA tensor. All cfgs
    share f_samp; each must be device_synth_supported."""
    import torch

    from . import _lib
    from .fitters import _torch_stream
    tab = synth_trial_table(cfgs, trial_nums, dynamic)
    f_samp = float(cfgs[0].f_samp)
    n = int(n_seconds * f_samp)
    out = torch.empty((len(cfgs), n), dtype=torch.float64, device="cuda")
    lib = _lib.load()
    _lib.check(lib.dfmi_synth_asd(tab.ctypes.data, len(cfgs), n, f_samp, out.data_ptr(), _lib.DFMI_MEM_DEVICE,
                                  _torch_stream()), "dfmi_synth_asd")
    return out


# --- counter-based snr-mode records (dfmi_synth_snr) ---------------------------
class SnrSpec:
    """Parameters of an unbounded snr-mode record whose sample i is a pure function of
    (spec, i) (include/dfmi.h dfmi_synth_snr): the signal of physics.py:493-518
    (is_dynamic=False) plus Philox4x32-10 white noise whose std follows
    physics.py:520-530 (signal power over one modulation cycle / 10^(snr/10)).

    Used where a record must be split over ranks (BASELINE config 4): every rank
    regenerates any segment — buffer 0 included — bit for bit."""

    def __init__(self, seed=1234, stream=0, f_samp=200000.0, f_mod=1000.0, amp=1.0, visibility=1.0, m=6.0,
                 phi=0.0, psi=0.0, snr_db=40.0):
        self.seed, self.stream = int(seed), int(stream)
        self.f_samp, self.f_mod = float(f_samp), float(f_mod)
        self.amp, self.visibility, self.m, self.phi, self.psi = (float(amp), float(visibility), float(m),
                                                                float(phi), float(psi))
        self.snr_db = snr_db
        ratio = self.f_samp / self.f_mod
        self.period = int(round(ratio)) if abs(ratio - round(ratio)) < 1e-9 and ratio < 2 ** 31 else 0

    def noise_std(self):
        if self.snr_db is None:
            return 0.0
        n = self.period if self.period > 0 else int(self.f_samp)
        t = np.arange(n) / self.f_samp
        clean = self.amp * (1 + self.visibility * np.cos(self.phi + self.m * np.cos(2 * np.pi * self.f_mod * t
                                                                                      + self.psi)))
        ac = clean - np.mean(clean)
        return float(np.sqrt(np.mean(ac ** 2) / 10 ** (self.snr_db / 10.0)))

    def params(self):
        from . import _lib
        return _lib.SnrParams(self.seed, self.stream, self.period, self.f_samp, self.f_mod, self.amp,
                              self.visibility, self.m, self.phi, self.psi, self.noise_std())


def synth_snr(spec: SnrSpec, idx0, n, out=None):
    """Samples [idx0, idx0 + n) of the record `spec` (dfmi_synth_snr, on the GPU).

    out: a contiguous float64 CUDA tensor (filled on its device's current stream) or
    None (returns a numpy array)."""
    from . import _lib
    lib = _lib.load()
    prm = spec.params()
    if out is not None and getattr(out, "is_cuda", False):
        import torch
        if out.dtype != torch.float64 or not out.is_contiguous() or out.numel() < n:
            raise ValueError("out must be a contiguous float64 CUDA tensor with >= n elements")
        with torch.cuda.device(out.device):
            _lib.check(lib.dfmi_synth_snr(prm, int(idx0), int(n), out.data_ptr(), _lib.DFMI_MEM_DEVICE,
                                          torch.cuda.current_stream(out.device).cuda_stream), "dfmi_synth_snr")
        return out
    host = np.empty(int(n), dtype=np.float64) if out is None else out
    _lib.check(lib.dfmi_synth_snr(prm, int(idx0), int(n), _lib.ptr(host), _lib.DFMI_MEM_HOST, None),
               "dfmi_synth_snr")
    return host
