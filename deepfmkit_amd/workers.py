"""Trial-level entry points (reference workers.py:8-189), kept as drop-in API.

`run_single_trial` / `run_efficiency_trial` keep the reference's
Configure-Simulate-Fit shape and call `DeepFitFramework.fit` (one tiny GPU
call per trial). `run_efficiency_trials` is the batched form (SURVEY.md §8f
item 2): it simulates every trial on the host and fits all of them in ONE
engine call — each trial is one record of one buffer, with its own seed.
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


def run_efficiency_trials(params_list):
    """Batched run_efficiency_trial: same results, one GPU call for all trials that
    share (f_samp, f_mod, n_seconds, ndata)."""
    from .physics import SignalGenerator
    out = np.full(len(params_list), np.nan)
    groups = {}
    for i, p in enumerate(params_list):
        lc = p["laser_config"]
        key = (float(lc.f_mod), float(p["n_seconds"]), int(p["ndata"]))
        groups.setdefault(key, []).append(i)
    for (f_mod, n_seconds, ndata), idx in groups.items():
        recs, guesses, f_samp = [], [], None
        for i in idx:
            p = params_list[i]
            cfg = DFMIObject("main_trial", p["laser_config"], p["ifo_config"])
            f_samp = cfg.f_samp
            raw = SignalGenerator().generate(cfg, n_seconds, mode="asd", trial_num=p["trial_num"])["main"]
            recs.append(np.asarray(raw.samples(), dtype=np.float64))
            guesses.append((1.6, p["m_true"], 0.0, 0.0))
        n = int(f_mod * n_seconds)
        R = int(f_samp / f_mod * n)
        nbuf = int(recs[0].size / R)
        if nbuf == 0:
            continue
        cols, _ = _fitters.nls_records([r[: nbuf * R] for r in recs], f_samp, f_mod, R, nbuf, ndata,
                                       np.array(guesses), parallel=False)
        m = np.asarray(cols[1]).reshape(len(idx), nbuf)[:, 0]
        out[np.array(idx)] = m
    return out
