"""Passes and time of the EKF parallel in time on the test set's hardest records (m = 9, phi = 1.3
and m = 4.3, psi = 0.3, phi = 0.7 fitted from init_m = 6; 50,000 samples, three channels in one
call) across block sizes and head lengths. One JSON line per setting."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def raw(dfm, m, seconds, trial, psi=0.0, phi=0.0):
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    laser.psi = psi
    ifo.phi = phi
    dfm.set_laser_df_for_effect(laser, ifo, m)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("p", laser, ifo, f_samp=200000.0))
    dff.simulate("p", n_seconds=seconds, mode="snr", snr_db=40.0, trial_num=trial)
    return np.ascontiguousarray(dff.raws["p"].samples(), dtype=np.float64)


def main():
    import torch  # noqa: F401
    import deepfmkit_amd as dfm
    from deepfmkit_amd import _lib
    lib = _lib.load()
    xs = [raw(dfm, 6.0, 0.25, 11), raw(dfm, 4.3, 0.25, 12, psi=0.3, phi=0.7), raw(dfm, 9.0, 0.25, 13, phi=1.3)]
    x = np.ascontiguousarray(np.concatenate(xs))
    n, nrec, R, nbuf = xs[0].size, len(xs), 4000, 12
    i4, p0, q = np.array([1.6, 6.0, 0.0, 0.0]), np.ones(5), np.array([1e-8, 1e-8, 1e-6, 1e-6, 1e-8])
    st = np.zeros((nrec, nbuf, 5))
    for head in (256, 512, 1024):
        for B in (16, 25, 32, 48, 64):
            _lib.check(lib.dfmi_set_tuning(b"ekf_pit_block", B), "tune")
            _lib.check(lib.dfmi_set_tuning(b"ekf_pit_head", head), "tune")
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                _lib.check(lib.dfmi_ekf_fit(_lib.ptr(x), nrec, n, n, _lib.ptr(i4), _lib.ptr(p0), _lib.ptr(q), None,
                                            2 * np.pi * 1000.0, 200000.0, R, nbuf, _lib.ptr(st), _lib.DFMI_MEM_HOST,
                                            None), "fit")
                ts.append(time.perf_counter() - t0)
            passes = (ctypes.c_int32 * nrec)()
            _lib.check(lib.dfmi_ekf_pit_passes(ctypes.cast(passes, ctypes.c_void_p), nrec), "passes")
            print(json.dumps({"head": head, "block": B, "passes": list(passes), "ms_host_incl": round(min(ts) * 1e3, 3)}),
                  flush=True)
    _lib.check(lib.dfmi_set_tuning(b"ekf_pit_block", 0), "tune")
    _lib.check(lib.dfmi_set_tuning(b"ekf_pit_head", 256), "tune")


if __name__ == "__main__":
    main()
