"""Trial-level entry points (reference workers.py:8-189), kept as drop-in API.

`run_single_trial` / `run_efficiency_trial` keep the reference's
Configure-Simulate-Fit shape and call `DeepFitFramework.fit` (one tiny GPU
call per trial). `run_efficiency_trials` is the batched form (SURVEY.md §8f
item 2): it generates every trial's record on the GPU (dfmi_synth_asd) and fits
all of them in ONE engine call — each trial is one record of one buffer, with
its own seed.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import scipy.constants as sc

from . import core as dfm
from . import fitters as _fitters
from .physics import DFMIObject, InterferometerConfig, LaserConfig


def calculate_ambiguity_boundary_point(params):
    """workers.py:8-42."""
    delta_f = params["delta_f"]
    delta_l = params["delta_l"]
    f0 = params["f0"]
    gi, gj = params["grid_i"], params["grid_j"]
    if delta_f == 0:
        return (gi, gj, float("inf"))
    err = -2 * np.pi * (delta_l / sc.c) * (f0 / delta_f)
    return (gi, gj, np.abs(err))


def run_single_trial(laser_config: LaserConfig, main_ifo_config: InterferometerConfig, fitter_method: str,
                     fitter_kwargs: Optional[dict] = None, witness_ifo_config: Optional[InterferometerConfig] = None,
                     n_seconds: Optional[float] = None, trial_num: int = 0):
    """workers.py:44-130: configure, simulate (asd mode), fit."""
    if fitter_kwargs is None:
        fitter_kwargs = {}
    dff = dfm.DeepFitFramework()
    main_label = "main_trial"
    main = DFMIObject(main_label, laser_config, main_ifo_config)
    dff.sims[main_label] = main
    witness_label = None
    if witness_ifo_config:
        witness_label = "witness_trial"
        dff.sims[witness_label] = DFMIObject(witness_label, laser_config, witness_ifo_config)
    if n_seconds is None:
        n_seconds = fitter_kwargs.get("n", main.fit_n) / laser_config.f_mod
    dff.simulate(main_label, n_seconds=n_seconds, witness_label=witness_label, trial_num=trial_num)
    if "wdfmi" in fitter_method:
        fitter_kwargs["witness_label"] = witness_label
    fitter_kwargs["verbose"] = False
    return dff.fit(main_label, method=fitter_method, **fitter_kwargs)


def run_efficiency_trial(params: dict) -> float:
    """workers.py:132-189: one single-buffer NLS fit, returns m."""
    laser_config = params["laser_config"]
    fitter_kwargs = {"n": int(laser_config.f_mod * params["n_seconds"]), "ndata": params["ndata"],
                     "init_m": params["m_true"], "parallel": False}
    fit_obj = run_single_trial(laser_config=laser_config, main_ifo_config=params["ifo_config"],
                               fitter_method="nls", fitter_kwargs=fitter_kwargs, n_seconds=params["n_seconds"],
                               trial_num=params["trial_num"])
    if fit_obj and fit_obj.m.size > 0:
        return fit_obj.m[0]
    return np.nan


class _TrialCfg:
    """The fields of DFMIObject("main_trial", laser, ifo) the device generator reads
    (run_single_trial's channel, default f_samp), without the object's set-up cost."""
    __slots__ = ("laser", "ifo", "f_samp")

    def __init__(self, laser, ifo):
        self.laser, self.ifo, self.f_samp = laser, ifo, _DEFAULT_F_SAMP


_DEFAULT_F_SAMP = DFMIObject("_", LaserConfig(), InterferometerConfig()).f_samp


def run_efficiency_trials(params_list, synth="device"):
    """Batched run_efficiency_trial: one GPU fit call for all trials that share
    (f_samp, f_mod, n_seconds, ndata), each trial a record with its own seed.

    synth="device": the trials' asd-mode records are generated on the GPU
    (physics.synthesize_asd_trials -> dfmi_synth_asd: numpy's RandomState stream and
    the exact-delay model restated; records within ~1e-15 of numpy's, the device's
    cos / sin / log being the only difference) and stay in HBM for the fit; trials the
    device generator does not cover (custom waveform) use the host generator.
    synth="host": the package's numpy generator for every trial (results then equal
    run_efficiency_trial's bit for bit)."""
    from .physics import SignalGenerator, device_synth_supported, synthesize_asd_trials
    if synth not in ("device", "host"):
        raise ValueError("synth must be 'device' or 'host'")
    out = np.full(len(params_list), np.nan)
    groups = {}
    for i, p in enumerate(params_list):
        lc = p["laser_config"]
        cfg = _TrialCfg(lc, p["ifo_config"]) if synth == "device" else DFMIObject("main_trial", lc, p["ifo_config"])
        dev = synth == "device" and device_synth_supported(cfg)
        if synth == "device" and not dev:
            cfg = DFMIObject("main_trial", lc, p["ifo_config"])
        key = (float(cfg.f_samp), float(lc.f_mod), float(p["n_seconds"]), int(p["ndata"]), dev)
        groups.setdefault(key, []).append((i, cfg))
    for (f_samp, f_mod, n_seconds, ndata, dev), members in groups.items():
        idx = [i for i, _ in members]
        guesses = np.array([(1.6, params_list[i]["m_true"], 0.0, 0.0) for i in idx])
        n = int(f_mod * n_seconds)
        R = int(f_samp / f_mod * n)
        N = int(n_seconds * f_samp)
        nbuf = int(N / R) if R > 0 else 0
        if nbuf == 0:
            continue  # the reference logs "nbuf is zero" and returns an empty fit -> nan
        if N % R != 0:
            # run_efficiency_trial raises here: _fit_sequential reshapes the whole
            # record with reshape(-1, R) (fitters.py:375)
            raise ValueError(f"cannot reshape array of size {N} into shape ({R})")
        if dev:
            x = synthesize_asd_trials([c for _, c in members], [params_list[i]["trial_num"] for i in idx], n_seconds)
            recs = x[:, : nbuf * R]
        else:
            recs = []
            for i, cfg in members:
                raw = SignalGenerator().generate(cfg, n_seconds, mode="asd", trial_num=params_list[i]["trial_num"])
                recs.append(np.asarray(raw["main"].samples(), dtype=np.float64)[: nbuf * R])
        cols, _ = _fitters.nls_records(recs, f_samp, f_mod, R, nbuf, ndata, guesses, parallel=False)
        m = cols[1].cpu().numpy() if hasattr(cols, "cpu") else np.asarray(cols[1])
        out[np.array(idx)] = m.reshape(len(idx), nbuf)[:, 0]
    return out
