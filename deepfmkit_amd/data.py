"""Raw and fit containers (reference data.py:16-309, hot-path subset).

`DeepRawObject.data` keeps the reference's shape — a pandas DataFrame with one
float64 column `ch0` — so code written against the reference keeps working. A
torch tensor already resident on the GPU is also accepted as `data` (the
device-resident path used by bench.py); `samples()` hands either form to the
engine without a copy.
"""
from __future__ import annotations

import numpy as np
import pandas as pd


class DeepRawObject:
    """One raw channel plus metadata (reference data.py:16-42)."""

    def __init__(self, data=None):
        self.raw_file = None
        self.label = None
        self.t0 = None
        self.f_samp = None
        self.f_mod = None
        self.sim = None
        self.data = pd.DataFrame()
        self.phi = None
        self.phi_sim = None
        self.phi_sim_downsamp = None
        self.f_noise = None
        self.l_noise = None
        self.a_noise = None
        self.df_noise = None
        if data is not None:
            if isinstance(data, np.ndarray):
                data = pd.DataFrame(np.asarray(data, dtype=np.float64).reshape(-1), columns=["ch0"])
            self.data = data

    def samples(self):
        """The channel's samples as a 1-D float64 array or device tensor (no copy)."""
        d = self.data
        if isinstance(d, pd.DataFrame):
            return d["ch0"].to_numpy() if "ch0" in d.columns else d.iloc[:, 0].to_numpy()
        if isinstance(d, pd.Series):
            return d.to_numpy()
        return d  # numpy array or torch tensor

    def n_samples(self):
        d = self.data
        return int(d.shape[0])


class DeepFitObject:
    """Fit results of one channel (reference data.py:121-208)."""

    def __init__(self):
        self.fit_file = None
        self.label = None
        self.n = None
        self.t0 = None
        self.R = None
        self.fs = None
        self.f_samp = None
        self.f_mod = None
        self.ndata = 10
        self.init_a = 1.6
        self.init_m = 6.0
        self.nbuf = None
        self.time = np.array([])
        self.ssq = np.array([])
        self.amp = np.array([])
        self.m = np.array([])
        self.tau = np.array([])
        self.phi = np.array([])
        self.psi = np.array([])
        self.dc = np.array([])

    def to_txt(self, filename):
        """fit_data text format (reference data.py:178-208), written by libdfmi's
        host writer in the reference's exact bytes (textio.write_fit)."""
        from . import textio
        textio.write_fit(self, filename)
