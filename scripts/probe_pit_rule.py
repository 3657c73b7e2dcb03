"""The EKF parallel-in-time stop rule (ekf_pit.h pit_decide) on the GPU: per record, the moves
d_k of every pass, the contraction d_k / d_{k-1}, the true distance of pass k's snapshots from
the scalar C oracle (oracle/csrc/ekf_scalar.c) with the rule switched off (ekf_pit_tol 99,
ekf_pit_seq 0, cap k), and what the default rule decides (passes, error, time). Then the
stress batches of tests/helpers/ekf_stress.py (pass histogram, sequential re-runs, worst error).
One JSON line per item on stdout."""
import collections
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "helpers"))
import ekf_stress as S  # noqa: E402

QD = np.array([1e-8, 1e-8, 1e-6, 1e-6, 1e-8])


def raw(dfm, m, seconds, trial, psi=0.0, phi=0.0):
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    laser.psi = psi
    ifo.phi = phi
    dfm.set_laser_df_for_effect(laser, ifo, m)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("p", laser, ifo, f_samp=200000.0))
    dff.simulate("p", n_seconds=seconds, mode="snr", snr_db=40.0, trial_num=trial)
    return np.ascontiguousarray(dff.raws["p"].samples(), dtype=np.float64)


def tune(lib, **kw):
    from deepfmkit_amd import _lib
    for k, v in kw.items():
        _lib.check(lib.dfmi_set_tuning(k.encode(), int(v)), "tune " + k)


DEFAULTS = dict(ekf_pit_passes=0, ekf_pit_first=5, ekf_pit_every=2, ekf_pit_tol=13, ekf_pit_stall=3,
                ekf_pit_trace=0, ekf_pit_seq=1, ekf_pit_block=0, ekf_pit_head=256, ekf_pit_measure=0)


def main():
    import deepfmkit_amd as dfm
    from deepfmkit_amd import _lib
    lib = _lib.load()
    cl = S.c_oracle()
    recs = {
        "config5_m6": (raw(dfm, 6.0, 2.0, 7), (1.6, 6.0, 0.0, 0.0), QD, None, 4000),
        "m9_phi13_init6": (raw(dfm, 9.0, 2.0, 13, phi=1.3), (1.6, 6.0, 0.0, 0.0), QD, None, 4000),
        "m43_tuned": (raw(dfm, 4.3, 1.0, 11, psi=0.3, phi=0.7), (1.6, 6.0, 0.0, 0.0),
                      np.array([1e-9, 1e-9, 1e-7, 1e-7, 1e-9]), 0.001, 4000),
        "m20_init6": (raw(dfm, 20.0, 1.0, 5), (1.6, 6.0, 0.0, 0.0), QD, None, 4000),
    }
    for name, (x, i4, qd, rvv, R) in recs.items():
        n = x.size
        nbuf = n // R
        x0 = np.array(list(i4) + [np.mean(x)])
        rv = np.array([np.var(x) if rvv is None else rvv])
        ref = S.c_states(cl, x, x0, rv[0], qd, R, nbuf)
        maxp = 20
        tune(lib, **DEFAULTS)
        tune(lib, ekf_pit_trace=1, ekf_pit_tol=99, ekf_pit_stall=1000, ekf_pit_seq=0, ekf_pit_passes=maxp,
             ekf_pit_first=maxp)
        errs = []
        for k in range(1, maxp + 1):
            tune(lib, ekf_pit_passes=k, ekf_pit_first=k)
            got, kname, passes = S.gpu_states(lib, x[None, :], x0[None, :], rv, qd, R, nbuf)
            errs.append(float(S.rel_err(got, ref[None])[0]))
        tr = np.empty(maxp)
        _lib.check(lib.dfmi_ekf_pit_trace(tr.ctypes.data, 1, maxp), "trace")
        tune(lib, ekf_pit_measure=1)
        S.gpu_states(lib, x[None, :], x0[None, :], rv, qd, R, nbuf)
        tr_ent = np.empty(maxp)
        _lib.check(lib.dfmi_ekf_pit_trace(tr_ent.ctypes.data, 1, maxp), "trace")
        tune(lib, ekf_pit_measure=0)
        rho = [None] + [float(tr[i] / tr[i - 1]) if np.isfinite(tr[i - 1]) and tr[i - 1] > 0 else None
                        for i in range(1, maxp)]
        tune(lib, **DEFAULTS)
        tune(lib, ekf_pit_trace=1)
        got, kname, passes = S.gpu_states(lib, x[None, :], x0[None, :], rv, qd, R, nbuf)
        trd = np.empty(256)
        _lib.check(lib.dfmi_ekf_pit_trace(trd.ctypes.data, 1, trd.size), "trace")
        tune(lib, ekf_pit_trace=0)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            S.gpu_states(lib, x[None, :], x0[None, :], rv, qd, R, nbuf)
            ts.append(time.perf_counter() - t0)
        seq_err = None
        tune(lib, ekf_pit=0)
        sq, kseq, _ = S.gpu_states(lib, x[None, :], x0[None, :], rv, qd, R, nbuf)
        seq_err = float(S.rel_err(sq, ref[None])[0])
        tune(lib, ekf_pit=1024)
        print(json.dumps({"record": name, "n": n, "moves": [None if not np.isfinite(v) else float(v) for v in tr],
                          "moves_entry": [None if not np.isfinite(v) else float(v) for v in tr_ent],
                          "rho": rho, "err_vs_c_at_pass": errs,
                          "default_rule": {"passes": int(passes[0]), "kernel": kname,
                                           "err_vs_c": float(S.rel_err(got, ref[None])[0]),
                                           "moves": [float(v) for v in trd[: abs(int(passes[0]))]],
                                           "ms_host_incl_min": round(min(ts) * 1e3, 3)},
                          "sequential": {"kernel": kseq, "err_vs_c": seq_err}}), flush=True)
    tune(lib, **DEFAULTS)
    hist = collections.Counter()
    n_ch = n_seq = 0
    worst = 0.0
    for bi, (n, nch, R) in enumerate(S.BATCHES):
        x, x0, rv, qd, meta = S.batch_inputs(bi, n, nch)
        nbuf = n // R
        tune(lib, ekf_pit_trace=1)
        t0 = time.perf_counter()
        got, kname, passes = S.gpu_states(lib, x, x0, rv, qd, R, nbuf)
        dt = time.perf_counter() - t0
        tr = np.empty((nch, 256))
        _lib.check(lib.dfmi_ekf_pit_trace(tr.ctypes.data, nch, tr.shape[1]), "trace")
        tune(lib, ekf_pit_trace=0, ekf_pit=0)
        t0 = time.perf_counter()
        sq, kseq, _ = S.gpu_states(lib, x, x0, rv, qd, R, nbuf)
        dts = time.perf_counter() - t0
        tune(lib, ekf_pit=1024)
        ref, sens = S.oracle_batch(cl, x, x0, rv, qd, R, nbuf, threads=16)
        err = S.rel_err(got, ref)
        err_seq = S.rel_err(sq, ref)
        hist.update(int(p) for p in passes)
        n_ch += nch
        n_seq += int((passes < 0).sum())
        worst = max(worst, float(err.max()))
        print(json.dumps({"batch": bi, "n": n, "channels": nch, "R": R, "kernel": kname, "s_host_incl": round(dt, 4),
                          "seq_kernel": kseq, "seq_s_host_incl": round(dts, 4),
                          "passes": [int(p) for p in passes], "err": [float(e) for e in err],
                          "err_seq": [float(e) for e in err_seq], "sens": [float(v) for v in sens],
                          "m": [float(v) for v in meta["m"]], "snr_db": [float(v) for v in meta["snr_db"]],
                          "init_dm": [float(v) for v in meta["init_dm"]],
                          "moves": [[None if not np.isfinite(v) else float(v) for v in tr[c, : abs(int(passes[c]))]]
                                    for c in range(nch)]}), flush=True)
    print(json.dumps({"stress_total": {"channels": n_ch, "sequential_reruns": n_seq,
                                       "pass_histogram": sorted(hist.items()), "max_rel_err_vs_c": worst}}),
          flush=True)


if __name__ == "__main__":
    main()
