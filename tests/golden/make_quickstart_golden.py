"""Golden fixtures of the reference quickstart's OWN fit, at its own size (run HERE only).

notebooks/0.0_quickstart.ipynb (cell 0) builds a 10 s, 200 kS/s snr-mode channel (40 dB) of a
laser modulated at 1 kHz with m_target = 10*3.14 through set_laser_df_for_effect on an
interferometer with arms 0.1 m / 0.3 m, then calls dff.fit(label, ndata=int(2*m_target)):
n = 20 (R = 4000), 500 buffers, ndata 62, parallel=True with n_cores = os.cpu_count(). This
script runs exactly that through the read-only reference (imported as tests/golden/make_golden.py
does) and records, for ndata 62 and 30:

  nb     the notebook's call as written (n_cores = os.cpu_count() of this container, recorded)
  seq    StandardNLSFitter._fit_sequential (parallel=False)             fitters.py:370-393
  c1     _fit_parallel with chunk size 1 (every buffer seeded by buffer 0) fitters.py:395-428
  par4   _fit_parallel with n_cores=4 (np.array_split chains)            fitters.py:395-428

plus the per-buffer QI at ndata 62 (calculate_quadratures + means, fit.py:18-66; the ndata-30 QI
are its first 30 harmonics) and the facade's tau. The input is NOT stored: the test regenerates it
with deepfmkit_amd.physics (the reference's snr-mode generator restated, physics.py:475-530) and
checks the SHA-256 recorded in quickstart.json.

Usage:  python tests/golden/make_quickstart_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _import_reference, sha  # noqa: E402

COLS = ("amp", "m", "phi", "psi", "dc", "ssq", "fitok")


def quickstart_sim(dfm):
    """Cell 0 of notebooks/0.0_quickstart.ipynb, steps 1-6, verbatim in effect."""
    dff = dfm.DeepFitFramework()
    laser = dfm.LaserConfig(label="main_laser")
    laser.f_mod = 1000
    ifo = dfm.InterferometerConfig(label="dynamic_ifo")
    ifo.ref_arml = 0.1
    ifo.meas_arml = 0.3
    m_target = 10 * 3.14
    dfm.set_laser_df_for_effect(laser, ifo, m_target)
    label = "dynamic_channel"
    dff.load_sim(dfm.DFMIObject(label=label, laser_config=laser, ifo_config=ifo, f_samp=200e3))
    dff.simulate(main_label=label, n_seconds=10, mode="snr", snr_db=40)
    return dff, label, m_target


def main():
    import pandas as pd
    import scipy
    dfm, rfit, rfitters = _import_reference()
    dff, label, m_target = quickstart_sim(dfm)
    raw = dff.raws[label]
    x = raw.data["ch0"].to_numpy()
    R, fs, nbuf = dff.fit_init(label, 20)
    out = {}
    meta = dict(generator="tests/golden/make_quickstart_golden.py",
                source="notebooks/0.0_quickstart.ipynb cell 0", numpy=np.__version__, scipy=scipy.__version__,
                m_target=m_target, f_mod=1000.0, f_samp=200000.0, n_seconds=10, snr_db=40, n=20, R=int(R),
                fs=float(fs), nbuf=int(nbuf), N=int(x.size), sha256=sha(x), df=float(dff.sims[label].laser.df),
                nb_n_cores=os.cpu_count(), ndata=[int(2 * m_target), 30])
    w0 = 2.0 * np.pi * raw.f_mod / raw.f_samp
    bufs = x[:nbuf * R].reshape(nbuf, R)
    nd = int(2 * m_target)
    qi = np.zeros((nbuf, 2 * nd))
    for b in range(nbuf):
        for h in range(nd):
            Q, I = rfit.calculate_quadratures(h, bufs[b], w0)
            qi[b, h] = Q.mean()
            qi[b, h + nd] = I.mean()
    out["qi62"] = qi
    for nd in meta["ndata"]:
        fobj = dff.fit(label, ndata=nd)  # the notebook's call (parallel, n_cores = os.cpu_count())
        df = dff.fits_df[f"{label}_nls"]  # core.py:471, 506-509
        for k in COLS:
            out[f"nd{nd}_nb_{k}"] = df[k].to_numpy()
        out[f"nd{nd}_nb_tau"] = np.asarray(fobj.tau)
        seq = rfitters.StandardNLSFitter({"n": 20}).fit(raw, parallel=False, ndata=nd)
        par4 = rfitters.StandardNLSFitter({"n": 20}).fit(raw, parallel=True, n_cores=4, ndata=nd)
        fitter = rfitters.StandardNLSFitter({"n": 20})
        first = fitter._fit_single_buffer(raw, 0, R, nd, np.array([1.6, 6.0, 0.0, 0.0]))
        seed = np.array([first["amp"], first["m"], first["phi"], first["psi"]])
        rows = [first]
        for b in range(1, nbuf):
            rows.extend(rfitters._process_fit_chunk((bufs[b:b + 1], seed, R, nd, raw.f_mod, raw.f_samp)))
        c1 = pd.DataFrame(rows)
        for mode, d in (("seq", seq), ("par4", par4), ("c1", c1)):
            for k in COLS:
                out[f"nd{nd}_{mode}_{k}"] = d[k].to_numpy()
        meta[f"nd{nd}_status_counts_nb"] = {str(s): int(c) for s, c in
                                            zip(*np.unique(out[f"nd{nd}_nb_fitok"], return_counts=True))}
        print(f"ndata {nd}: buffer 0 status {int(out[f'nd{nd}_c1_fitok'][0])}, m {out[f'nd{nd}_c1_m'][:3]}", flush=True)
    np.savez_compressed(os.path.join(HERE, "quickstart.npz"), **out)
    with open(os.path.join(HERE, "quickstart.json"), "w") as f:
        json.dump(meta, f, indent=1)


if __name__ == "__main__":
    main()
