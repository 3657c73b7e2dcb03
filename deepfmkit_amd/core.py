"""DeepFitFramework — the reference's drop-in facade (core.py:22-588), hot-path subset.

Kept: the containers (raws, sims, fits, fits_df), simulate (snr mode; asd mode
for zero/white noise), new_sim / load_sim, create_witness_channel, fit_init,
fit (strategy dispatch, tau column, DeepFitObject), fit_many — several
equal-length channels fitted as ONE GPU batch (config 3) — and the text formats:
parse_header, load_raw, load_fit, to_txt (core.py:119-174, 259-332; parsed and
written by libdfmi's host code, deepfmkit_amd/textio.py).

Out of scope (SURVEY.md §2 "OUT"): LPSD, plotting.
"""
from __future__ import annotations

import logging
import time

import numpy as np
import pandas as pd
import scipy.constants as sc

from . import fitters as _fitters
from .data import DeepFitObject
from .physics import DFMIObject, InterferometerConfig, SignalGenerator

log = logging.getLogger(__name__)


_time_axes = {}


def _time_axis(nbuf, fs):
    """core.py:515: np.arange(0, nbuf / fs, 1 / fs), formed once per (nbuf, fs) and handed out
    as a fresh copy (the caller owns its array, as with the reference's)."""
    key = (int(nbuf), float(fs))
    t = _time_axes.get(key)
    if t is None:
        if len(_time_axes) > 64:
            _time_axes.clear()
        t = _time_axes[key] = np.arange(0, nbuf / fs, 1.0 / fs)
    return t.copy()


def vectorized_downsample(signal, R):
    """dsp.py:3-55: boxcar mean over blocks of R (used for phi_sim only)."""
    if not isinstance(R, int) or R <= 0:
        return np.array([])
    signal = np.asarray(signal)
    n = (len(signal) // R) * R
    if n == 0:
        return np.array([])
    return signal[:n].reshape(-1, R).mean(axis=1)


class DeepFitFramework:
    def __init__(self, raw_file=None, fit_file=None, raw_labels=None, fit_labels=None):
        self.raw_file = raw_file
        self.fit_file = fit_file
        self.lasers = {}
        self.ifos = {}
        self.sims = {}
        self.raws = {}
        self.fits = {}
        self.fits_df = {}
        self.channr = None
        self.n = None
        self.t0 = None
        self.R = None
        self.fs = None
        self.f_samp = None
        self.f_mod = None
        self.ndata = 10
        self.init_a = 1.6
        self.init_m = 6.0
        if self.raw_file is not None:
            self.load_raw(labels=raw_labels)
        if self.fit_file is not None:
            self.load_fit(labels=fit_labels)

    # --- text formats (core.py:119-174, 259-332) --------------------------------
    def to_txt(self, filepath="./", labels=None):
        """core.py:119-127: one fit_data file per fit, named <filepath><label>.txt."""
        for label in (labels if labels is not None else list(self.fits)):
            self.fits[label].to_txt(filepath + self.fits[label].label + ".txt")

    def parse_header(self, file_select="raw"):
        """core.py:129-174."""
        from . import textio
        if file_select == "raw":
            h = textio.parse_header(self.raw_file, textio.RAW)
        elif file_select == "fit":
            h = textio.parse_header(self.fit_file, textio.FIT)
        else:
            log.error("No files specified !!")
            return
        for k, v in h.items():
            setattr(self, k, v)

    def load_raw(self, raw_file=None, labels=None, device=None):
        """core.py:259-286: one DeepRawObject per channel (column). With `device`
        the samples go straight to that GPU (pinned staging) as the raw's data."""
        from . import textio
        from .data import DeepRawObject
        if raw_file is not None:
            self.raw_file = raw_file
        if self.raw_file is None:
            log.error("No raw file specified !!")
            return
        self.parse_header(file_select="raw")
        if labels is None:
            labels = [self.raw_file + "_ch" + str(c) for c in range(self.channr)]
        else:
            assert len(labels) == self.channr
        _, chans = textio.read_raw(self.raw_file, device=device)
        for c in range(self.channr):
            if device is None:
                import pandas as pd
                raw = DeepRawObject(data=pd.DataFrame({"ch" + str(c): chans[c]}))
            else:
                raw = DeepRawObject(data=chans[c])
            raw.raw_file = self.raw_file
            raw.label = labels[c]
            raw.t0 = self.t0
            raw.f_samp = self.f_samp
            raw.f_mod = self.f_mod
            self.raws[raw.label] = raw

    def load_fit(self, fit_file=None, labels=None):
        """core.py:288-332 (labels default to <raw_file>_ch<c>, as the reference: a
        framework without a raw file raises the same TypeError)."""
        from . import textio
        if fit_file is not None:
            self.fit_file = fit_file
        if self.fit_file is None:
            log.error("No fit file specified !!")
            return
        self.parse_header(file_select="fit")
        if labels is None:
            labels = [self.raw_file + "_ch" + str(c) for c in range(self.channr)]
        else:
            assert len(labels) == self.channr
        _, data = textio.read_fit(self.fit_file)
        for k in range(self.channr):
            fit = DeepFitObject()
            fit.nbuf = data.shape[2]
            fit.n, fit.t0, fit.R, fit.fs = self.n, self.t0, self.R, self.fs
            fit.f_samp, fit.f_mod = self.f_samp, self.f_mod
            fit.ndata, fit.init_a, fit.init_m = self.ndata, self.init_a, self.init_m
            fit.ssq, fit.amp, fit.m, fit.phi, fit.psi, fit.dc = (data[k, i].copy() for i in range(6))
            fit.time = np.arange(0, fit.nbuf / self.fs, 1.0 / self.fs)
            fit.label = labels[k]
            self.fits[labels[k]] = fit

    # --- simulation ---------------------------------------------------------
    def load_sim(self, sim):
        self.sims[sim.label] = sim

    def new_sim(self, label=None):
        if label is None:
            from datetime import datetime
            label = datetime.now().strftime("%Y%m%d_%H%M%S")
        from .physics import LaserConfig
        sim = DFMIObject(label=label, laser_config=LaserConfig(), ifo_config=InterferometerConfig())
        self.sims[sim.label] = sim
        return label

    def simulate(self, main_label, n_seconds, mode="asd", witness_label=None, snr_db=None, trial_num=0,
                 verbose=False):
        """core.py:176-243."""
        t0 = time.time()
        if main_label not in self.sims:
            log.error(f"Main simulation label '{main_label}' not found!")
            return
        main_config = self.sims[main_label]
        witness_config = None
        if witness_label:
            if witness_label not in self.sims:
                log.error(f"Witness simulation label '{witness_label}' not found!")
                return
            witness_config = self.sims[witness_label]
        chans = SignalGenerator().generate(main_config=main_config, n_seconds=n_seconds, mode=mode,
                                           trial_num=trial_num, witness_config=witness_config, snr_db=snr_db)
        if not chans:
            log.error("Simulation failed to generate data.")
            return
        for _, raw in chans.items():
            self.raws[raw.label] = raw
        main_config.simtime = time.time() - t0

    def create_witness_channel(self, main_channel_label, witness_channel_label, m_witness=None,
                               delta_l_witness=None):
        """core.py:519-588: a static witness sharing the main channel's laser."""
        if main_channel_label not in self.sims:
            raise KeyError(f"Main channel '{main_channel_label}' not found in framework.")
        if delta_l_witness is not None and m_witness is not None:
            raise ValueError("Please specify either delta_l_witness or m_witness, but not both.")
        main = self.sims[main_channel_label]
        laser = main.laser
        if m_witness is None and delta_l_witness is None:
            m_target = 0.1
        elif m_witness is not None:
            m_target = m_witness
        else:
            m_target = (2 * np.pi * laser.df * delta_l_witness) / sc.c
        ifo = InterferometerConfig(label=f"{witness_channel_label}_ifo")
        ifo.arml_mod_amp = 0.0
        ifo.arml_mod_n = 0.0
        if laser.df == 0:
            raise ValueError("Cannot set 'm_witness' when laser 'df' is zero.")
        dl = (m_target * sc.c) / (2 * np.pi * laser.df)
        ifo.ref_arml = 0.01
        ifo.meas_arml = ifo.ref_arml + dl
        f0 = sc.c / laser.wavelength
        static_phase = (2 * np.pi * f0 * dl) / sc.c
        ifo.phi = ((np.pi / 2.0) + static_phase) % (2 * np.pi)
        w = DFMIObject(label=witness_channel_label, laser_config=laser, ifo_config=ifo, f_samp=main.f_samp)
        w.fit_n = main.fit_n
        self.sims[witness_channel_label] = w
        return w

    # --- fitting ------------------------------------------------------------
    def fit_init(self, label, n):
        """core.py:390-422."""
        raw = self.raws[label]
        R = int(raw.f_samp / raw.f_mod * n)
        fs = raw.f_samp / R
        nbuf = int(raw.n_samples() / R)
        if nbuf == 0:
            log.error("Check buffer size !! Calculated nbuf is zero.")
        return R, fs, nbuf

    def _n_cycles(self, raw, main_label, kwargs):
        n = kwargs.get("n")
        if n is None:
            sim = self.sims.get(raw.sim.label if raw.sim else main_label)
            n = sim.fit_n if sim else 20
        return n

    def fit(self, main_label, method="nls", fit_label=None, **kwargs):
        """core.py:424-517: strategy dispatch -> DataFrame -> DeepFitObject."""
        _fitters.mark("fit")
        fitter_map = _fitters.FITTER_MAP
        if method not in fitter_map:
            log.error(f"Unknown fit method: '{method}'. Available: {list(fitter_map.keys())}")
            return
        if main_label not in self.raws:
            log.error(f"Invalid raw data label: '{main_label}' !!")
            return
        raw = self.raws[main_label]
        if fit_label is None:
            fit_label = f"{main_label}_{method}"
        n = self._n_cycles(raw, main_label, kwargs)
        R, fs, nbuf = self.fit_init(main_label, n)
        if getattr(raw, "phi_sim", None) is not None and len(raw.phi_sim) > 0:
            raw.phi_sim_downsamp = vectorized_downsample(raw.phi_sim, R)
        fit_config = {"n": n}
        fitter_args = {"main_raw": raw}
        if "wdfmi" in method:  # core.py:486-490 (hwdfmi included)
            witness_label = kwargs.get("witness_label")
            if not witness_label or witness_label not in self.raws:
                log.error(f"W-DFMI method '{method}' requires a valid 'witness_label'.")
                return
            fitter_args["witness_raw"] = self.raws[witness_label]
        fitter = fitter_map[method](fit_config)
        df = fitter.fit(**fitter_args, **kwargs)
        if df is None or df.empty:
            log.error(f"{fitter_map[method].__name__} returned no results.")
            return None
        # the package's own NLS fitter returns frame_from's frame untouched: its column arrays
        # can be used as they are (any other fitter's frame is read through pandas)
        known = _fitters.frame_arrays(df) if type(fitter) is _fitters.StandardNLSFitter else None
        return self._finish(fit_label, main_label, raw, method, df, n, R, fs, nbuf, known)

    def _finish(self, fit_label, main_label, raw, method, df, n, R, fs, nbuf, known=None):
        arrays, with_tau = known if known is not None else (None, None)
        cols = dict(arrays) if arrays is not None else {k: df[k].to_numpy() for k in df.columns}
        if method == "nls" and with_tau is not None:
            df, cols["tau"] = with_tau  # the same columns with tau, formed by the fitter (frame_from)
        elif method in ("nls", "ekf"):
            # core.py:506-509: df['tau'] = df['m'] / (2 pi df) (0.0 without a sim). The column is
            # appended by rebuilding the frame over the same column arrays (pandas' __setitem__
            # would copy the array in), same columns, order and dtypes
            m = cols["m"]
            cols["tau"] = m / (2 * np.pi * raw.sim.laser.df) if raw.sim else np.zeros(m.shape[0])
            df = pd.DataFrame(cols, copy=False)
        _fitters.mark("tau")
        self.fits_df[fit_label] = df
        fit = DeepFitObject()
        # core.py:511-514 records ndata/init_a/init_m as 0 in the fit object
        fit.n, fit.R, fit.fs, fit.nbuf, fit.ndata, fit.init_a, fit.init_m = n, R, fs, nbuf, 0, 0, 0
        fit.t0, fit.f_samp, fit.f_mod = raw.t0, raw.f_samp, raw.f_mod
        for k in ("ssq", "amp", "m", "tau", "phi", "psi", "dc"):
            setattr(fit, k, cols[k] if k in cols else df[k].to_numpy())
        _fitters.mark("columns")
        fit.time = _time_axis(fit.ssq.shape[0], fit.fs)
        fit.label = fit_label
        self.fits[fit_label] = fit
        _fitters.mark("fitobj")
        return fit

    def fit_many(self, labels, method="nls", **kwargs):
        """Fit several channels in ONE engine call (lane/segment batch across channels).

        Equivalent to `for l in labels: self.fit(l, method, **kwargs)` (which is how
        notebooks/0.1_quickstart-2-ch fits its two channels), including the fit labels
        f"{label}_{method}" under which self.fits / self.fits_df store the results; channels
        that share f_samp, f_mod and length go through one engine call. Raises fit()'s
        ValueError when the record length is not a multiple of R (fitters.py:375, 412).
        Returns {label: DeepFitObject}."""
        raws = [self.raws[l] for l in labels]
        r0 = raws[0]
        if any(r.f_samp != r0.f_samp or r.f_mod != r0.f_mod or r.n_samples() != r0.n_samples() for r in raws):
            return {l: self.fit(l, method=method, **kwargs) for l in labels}
        n = self._n_cycles(r0, labels[0], kwargs)
        R, fs, nbuf = self.fit_init(labels[0], n)
        out = {}
        if method == "ekf":
            states = _fitters.ekf_records(raws, n, **{k: v for k, v in kwargs.items() if k != "n"})
            for l, raw, st in zip(labels, raws, states):
                import pandas as pd
                df = pd.DataFrame({"amp": st[:, 0], "m": st[:, 1], "phi": st[:, 2], "psi": st[:, 3], "dc": st[:, 4],
                                   "ssq": np.zeros(nbuf), "fitok": np.ones(nbuf, dtype=int)})
                out[l] = self._finish(f"{l}_{method}", l, raw, method, df, n, R, fs, nbuf)
            return out
        if method != "nls":
            return {l: self.fit(l, method=method, **kwargs) for l in labels}
        ndata = int(kwargs.get("ndata", 10))
        N = r0.n_samples()
        if N % R != 0:
            raise ValueError(f"cannot reshape array of size {N} into shape ({R})")
        parallel = kwargs.get("parallel", True)
        g = (kwargs.get("init_a", 1.6), kwargs.get("init_m", 6.0), 0.0, kwargs.get("init_psi", 0.0))
        cols, ok = _fitters.nls_records([r.samples() for r in raws], r0.f_samp, r0.f_mod, R, nbuf, ndata, g,
                                        parallel=parallel, n_cores=kwargs.get("n_cores") if parallel else None)
        df_all = _fitters.frame_from(cols, ok)
        for i, (l, raw) in enumerate(zip(labels, raws)):
            df = df_all.iloc[i * nbuf:(i + 1) * nbuf].reset_index(drop=True)
            out[l] = self._finish(f"{l}_{method}", l, raw, method, df, n, R, fs, nbuf)  # fit()'s default label
        return out
