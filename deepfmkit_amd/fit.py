"""NLS numerics front-end (mirror of the reference fit.py module surface).

The module-level constants have the reference's names and defaults
(fit.py:5-16); like the reference, callers may overwrite them at run time
(notebooks/0.0_benchmark.ipynb cell 1 does) — every engine call reads their
CURRENT values into the dfmi_lm_config it passes to libdfmi.

Batched entry points (all arithmetic runs in the HIP kernels of libdfmi.so):
  demodulate(buffers, ndata, w0)   -> (QI (nseg, 2*ndata), dc)   fit.py:18-66 + means
  fit_batch(ndata, QI, guess)       -> (status, p, ssq)           fit.py:322-361 per row
  fit(ndata, data, parm)            -> (status, p, ssq)           fit.py:322 single segment
"""
from __future__ import annotations

import numpy as np

from . import _lib

NPARMS = 4
MAXDATA = 40
MAX_LMA_STEPS = 100
LMA_CONVERGENCE_IMPROVE = 1e-9
LMA_CONVERGENCE_PARAM_CHANGE = 1e-9
FITOK_THRESHOLD = 1e-3
M_GRID_MIN = 5.0
M_GRID_MAX = 30.0
M_GRID_STEP = 0.5
BESSEL_AMP_THRESHOLD = 0.05
SINCOS_AMP_THRESHOLD = 0.1
LAMBDA_LADDER = (0.0, 1e-7, 1e-5, 1e-3, 1e-1, 1.0, 10.0, 100.0)  # fit.py:222
MIN_STEP_NORM = 1e-15  # fit.py:230


_cfg_cache = {}


def lm_config() -> _lib.LMConfig:
    """dfmi_lm_config from the module globals as they are NOW (built once per distinct set of
    values: a caller that changes a constant gets a new struct on its next call)."""
    key = (MAX_LMA_STEPS, tuple(LAMBDA_LADDER), MIN_STEP_NORM, LMA_CONVERGENCE_IMPROVE, LMA_CONVERGENCE_PARAM_CHANGE,
           FITOK_THRESHOLD, M_GRID_MIN, M_GRID_MAX, M_GRID_STEP, BESSEL_AMP_THRESHOLD, SINCOS_AMP_THRESHOLD)
    cfg = _cfg_cache.get(key)
    if cfg is None:
        cfg = _cfg_cache[key] = _lm_config_build()
    return cfg


def _lm_config_build() -> _lib.LMConfig:
    cfg = _lib.LMConfig()
    cfg.max_lma_steps = int(MAX_LMA_STEPS)
    lad = tuple(LAMBDA_LADDER)
    if len(lad) > _lib.MAX_LAMBDA:
        raise ValueError(f"at most {_lib.MAX_LAMBDA} damping values")
    cfg.n_lambda = len(lad)
    for i, v in enumerate(lad):
        cfg.lambdas[i] = float(v)
    cfg.min_step_norm = float(MIN_STEP_NORM)
    cfg.conv_improve = float(LMA_CONVERGENCE_IMPROVE)
    cfg.conv_param_change = float(LMA_CONVERGENCE_PARAM_CHANGE)
    cfg.fitok_threshold = float(FITOK_THRESHOLD)
    cfg.m_grid_min = float(M_GRID_MIN)
    cfg.m_grid_max = float(M_GRID_MAX)
    cfg.m_grid_step = float(M_GRID_STEP)
    cfg.bessel_amp_threshold = float(BESSEL_AMP_THRESHOLD)
    cfg.sincos_amp_threshold = float(SINCOS_AMP_THRESHOLD)
    return cfg


def demodulate(buffers, ndata: int, w0: float, period: int = 0):
    """QI of every row of `buffers` (nseg, R) float64 -> (QI (nseg, 2*ndata), dc (nseg,)).

    QI row layout is the reference's [Q_1..Q_ndata, I_1..I_ndata] (fitters.py:45-49)."""
    lib = _lib.load()
    x = np.ascontiguousarray(buffers, dtype=np.float64)
    if x.ndim != 2:
        raise ValueError("buffers must be (nseg, R)")
    nseg, R = x.shape
    qi_cm = np.empty((2 * ndata, nseg))
    dc = np.empty(nseg)
    _lib.check(lib.dfmi_demod(_lib.ptr(x), nseg, R, R, ndata, float(w0), int(period), _lib.ptr(qi_cm),
                              _lib.ptr(dc), _lib.DFMI_MEM_HOST, None), "dfmi_demod")
    return np.ascontiguousarray(qi_cm.T), dc


def fit_batch(ndata: int, qi, guess):
    """fit.fit (fit.py:322-361) applied to every row of qi (nseg, 2*ndata), each row
    seeded by its own guess row (nseg, 4) or by one shared guess (4,)."""
    lib = _lib.load()
    qi = np.asarray(qi, dtype=np.float64)
    if qi.ndim == 1:
        qi = qi[None, :]
    nseg = qi.shape[0]
    if qi.shape[1] != 2 * ndata:
        raise ValueError("qi rows must have 2*ndata entries")
    qi_cm = np.ascontiguousarray(qi.T)
    g = np.asarray(guess, dtype=np.float64)
    if g.ndim == 1:
        g = np.broadcast_to(g, (nseg, 4))
    g = np.ascontiguousarray(g)
    params = np.empty((4, nseg))
    ssq = np.empty(nseg)
    status = np.empty(nseg, dtype=np.int32)
    cfg = lm_config()
    _lib.check(lib.dfmi_lm(_lib.ptr(qi_cm), nseg, ndata, _lib.ptr(g), 1, nseg, cfg, _lib.ptr(params),
                           _lib.ptr(ssq), _lib.ptr(status), _lib.DFMI_MEM_HOST, None), "dfmi_lm")
    return status, np.ascontiguousarray(params.T), ssq


def fit(ndata, data, parm):
    """Single-segment form of the reference entry point fit.fit(ndata, data, parm)."""
    st, p, ssq = fit_batch(ndata, np.asarray(data, dtype=np.float64)[None, :], np.asarray(parm, dtype=np.float64))
    return int(st[0]), p[0].copy(), float(ssq[0])
