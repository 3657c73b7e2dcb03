"""Edge-case parity fixtures from the reference DeepFMKit (run HERE only; the reference
never travels to the GPU box): records with erasures / non-finite samples, fitted by the
reference's own StandardNLSFitter (fitters.py:330-447).

One snr-mode record (m = 6, 40 dB, f_mod 1 kHz, 200 kS/s, n = 4 cycles: R = 800,
10 buffers), then five defective copies:
  nan_mid     one NaN sample in buffer 3
  inf_mid     one +inf sample in buffer 5
  zero_buf    buffer 2 all zeros (a -> 0: fit.py:126-128)
  nan_seed    one NaN sample in buffer 0 (the seed of every parallel chunk)
  spike       one sample + 1e3 in buffer 4
Each through the sequential path, the parallel path with chunk size 1 (every buffer
seeded from buffer 0) and the reference's parallel path with n_cores = 4. Inputs are
stored (data only) in edge_records.npz next to the outputs.

Usage:  python tests/golden/make_edge_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _import_reference, df_to_arrays  # noqa: E402

R_CYC = 4
CASES = ("clean", "nan_mid", "inf_mid", "zero_buf", "nan_seed", "spike")


def defect(x, R, case):
    y = x.copy()
    if case == "nan_mid":
        y[3 * R + 17] = np.nan
    elif case == "inf_mid":
        y[5 * R + 100] = np.inf
    elif case == "zero_buf":
        y[2 * R:3 * R] = 0.0
    elif case == "nan_seed":
        y[10] = np.nan
    elif case == "spike":
        y[4 * R + 5] += 1e3
    return y


def main():
    import warnings

    import pandas as pd
    from scipy.constants import c, pi
    dfm, rfit, rfitters = _import_reference()
    warnings.simplefilter("ignore")  # numpy RuntimeWarnings of the non-finite cases
    laser = dfm.LaserConfig(label="laser")
    laser.f_mod = 1000.0
    ifo = dfm.InterferometerConfig(label="ifo")
    laser.df = (6.0 * c) / (2 * pi * abs(ifo.meas_arml - ifo.ref_arml))
    sim = dfm.DFMIObject(label="edge", laser_config=laser, ifo_config=ifo, f_samp=200000)
    dff = dfm.DeepFitFramework()
    dff.load_sim(sim)
    dff.simulate("edge", n_seconds=0.04, mode="snr", snr_db=40.0, trial_num=3)
    raw = dff.raws["edge"]
    x0 = raw.data["ch0"].to_numpy().copy()
    R, _, nbuf = dff.fit_init("edge", R_CYC)
    out = {"R": np.int64(R), "nbuf": np.int64(nbuf), "n": np.int64(R_CYC), "f_samp": raw.f_samp,
           "f_mod": raw.f_mod}
    nd = 10
    for case in CASES:
        x = defect(x0, R, case)
        raw.data = pd.DataFrame({"ch0": x})
        out[f"{case}_x"] = x
        seq = rfitters.StandardNLSFitter({"n": R_CYC}).fit(raw, parallel=False, ndata=nd)
        for k, v in df_to_arrays(seq).items():
            out[f"{case}_seq_{k}"] = v
        fitter = rfitters.StandardNLSFitter({"n": R_CYC})
        first = fitter._fit_single_buffer(raw, 0, R, nd, np.array([1.6, 6.0, 0.0, 0.0]))
        seed = np.array([first["amp"], first["m"], first["phi"], first["psi"]])
        bufs = x[:nbuf * R].reshape(nbuf, R)
        rows = [first]
        for b in range(1, nbuf):
            rows.extend(rfitters._process_fit_chunk((bufs[b:b + 1], seed, R, nd, raw.f_mod, raw.f_samp)))
        for k, v in df_to_arrays(pd.DataFrame(rows)).items():
            out[f"{case}_c1_{k}"] = v
        par = rfitters.StandardNLSFitter({"n": R_CYC}).fit(raw, parallel=True, n_cores=4, ndata=nd)
        for k, v in df_to_arrays(par).items():
            out[f"{case}_par4_{k}"] = v
        print(case, "seq fitok", out[f"{case}_seq_fitok"], "c1 fitok", out[f"{case}_c1_fitok"])
    np.savez_compressed(os.path.join(HERE, "edge_records.npz"), **out)


if __name__ == "__main__":
    main()
