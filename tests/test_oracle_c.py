"""The oracle's C restatements against the numpy oracle (pinned to the reference's golden
vectors): EKFFitter's loop (oracle/csrc/ekf_scalar.c, the scalar CPU baseline of config 5):
same states to fp64 rounding; the NLS readout (oracle/csrc/nls_scalar.c, bench.py's second CPU
baseline): status equal, status-0 parameters within 1e-9."""
import ctypes
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "oracle", "libekf_scalar.so")


def test_ekf_scalar_c_matches_oracle():
    if not os.path.exists(SO):
        pytest.skip("oracle C restatement not built (run __graft_entry__.build())")
    import deepfmkit_amd as dfm
    from oracle import nls_oracle as O
    laser = dfm.LaserConfig()
    ifo = dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("e", laser, ifo, f_samp=200000.0))
    dff.simulate("e", n_seconds=0.04, mode="snr", snr_db=40.0, trial_num=2)
    x = np.asarray(dff.raws["e"].samples(), dtype=np.float64)
    ref = O.ekf_record(x, 200000.0, 1000.0, 20)
    lib = ctypes.CDLL(SO)
    P = ctypes.c_void_p
    lib.ekf_scalar.argtypes = [P, ctypes.c_int64, P, P, P, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                               ctypes.c_int64, ctypes.c_int64, P]
    x0 = np.array([1.6, 6.0, 0.0, 0.0, np.mean(x)])
    p0, qd = np.ones(5), np.array([1e-8, 1e-8, 1e-6, 1e-6, 1e-8])  # held: ctypes gets raw pointers
    out = np.zeros((ref.shape[0], 5))
    lib.ekf_scalar(x.ctypes.data, x.size, x0.ctypes.data, p0.ctypes.data, qd.ctypes.data, float(np.var(x)),
                   2 * np.pi * 1000.0, 200000.0, 4000, ref.shape[0], out.ctypes.data)
    assert np.max(np.abs(out - ref)) <= 1e-12


def test_nls_scalar_c_matches_oracle():
    """Chunk-size-1 parallel semantics (fitters.py:395-428 with n_cores >= nbuf - 1) on the
    reference's clean edge record and on a 200-segment config-2-shaped snr record, 1 and
    4 OpenMP threads (same results)."""
    so = os.path.join(ROOT, "oracle", "libnls_scalar.so")
    if not os.path.exists(so):
        pytest.skip("oracle C restatement not built (run __graft_entry__.build())")
    import deepfmkit_amd as dfm
    from oracle import nls_oracle as O
    lib = ctypes.CDLL(so)
    P = ctypes.c_void_p
    lib.nls_scalar_record.argtypes = [P, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_double, P,
                                      ctypes.c_int, P]
    d = np.load(os.path.join(ROOT, "tests", "golden", "edge_records.npz"))
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    raw = dfm.SignalGenerator().generate(dfm.DFMIObject("c", laser, ifo, f_samp=200000.0), 200 * 4000 / 200000.0,
                                         mode="snr", snr_db=40.0, trial_num=5)["main"]
    cases = [(d["clean_x"], float(d["f_samp"]), float(d["f_mod"]), int(d["n"])),
             (np.asarray(raw.samples(), dtype=np.float64), 200000.0, 1000.0, 20)]
    for x, fs, fm, n in cases:
        R, _, nb = O.buffer_params(x.size, fs, fm, n)
        ref = O.fit_record_parallel(x, fs, fm, n, n_cores=max(1, nb - 1))
        for th in (1, 4):
            out = np.zeros((nb, 7))
            g = np.array([1.6, 6.0, 0.0, 0.0])
            assert lib.nls_scalar_record(x.ctypes.data, nb, R, 10, 2 * np.pi * fm / fs, g.ctypes.data, th,
                                         out.ctypes.data) == 0
            np.testing.assert_array_equal(out[:, 6], ref[:, 6])
            ok = ref[:, 6] == 0
            for j in range(4):
                dj = np.abs(out[ok, j] - ref[ok, j])
                if j == 2:
                    dj = np.abs((dj + np.pi) % (2 * np.pi) - np.pi)
                assert dj.max() <= 1e-9, (j, dj.max())
            assert np.abs(out[:, 4] - ref[:, 4]).max() <= 1e-13


@pytest.mark.parametrize("group", ["10", "5", "20", "30", "62", "edge10"])
def test_lm_scalar_c_on_reference_lm_vectors(lm_npz, group):
    """The C restatement's fit.fit (lm_scalar_fit) on the reference's own LM vectors
    (tests/golden/lm_vectors.npz): the same gates as the GPU (conftest.check_lm_group)."""
    from conftest import check_lm_group
    so = os.path.join(ROOT, "oracle", "libnls_scalar.so")
    if not os.path.exists(so):
        pytest.skip("oracle C restatement not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(so)
    P = ctypes.c_void_p
    lib.lm_scalar_fit.argtypes = [P, ctypes.c_int64, ctypes.c_int, P, ctypes.c_int, P]
    qi = np.ascontiguousarray(lm_npz[f"g{group}_qi"])
    g = np.ascontiguousarray(lm_npz[f"g{group}_guess"])
    n, nd = qi.shape[0], qi.shape[1] // 2
    out = np.zeros((n, 6))
    assert lib.lm_scalar_fit(qi.ctypes.data, n, nd, g.ctypes.data, 4, out.ctypes.data) == 0
    check_lm_group(lm_npz, group, out[:, 5].astype(int), out[:, :4], out[:, 4])


@pytest.mark.parametrize("run", ["c5_default", "c5_tuned"])
def test_ekf_scalar_c_full_length_vs_reference(run):
    """The scalar C restatement (config 5's CPU baseline) against the reference's own
    EKFFitter states at full length (2 s = 400,000 samples, tests/golden/ekf_full.npz,
    default and tuned Q / R): 1e-12 on every snapshot."""
    if not os.path.exists(SO):
        pytest.skip("oracle C restatement not built (run __graft_entry__.build())")
    import json
    from conftest import make_record, sha
    with open(os.path.join(ROOT, "tests", "golden", "manifest.json")) as f:
        e = {r["name"]: r for r in json.load(f)["ekf_full"]}[run]
    d = np.load(os.path.join(ROOT, "tests", "golden", "ekf_full.npz"))
    x = np.ascontiguousarray(make_record(e).raws[run].samples(), dtype=np.float64)
    assert sha(x) == e["sha256"]
    kw = e["fit_kwargs"]
    lib = ctypes.CDLL(SO)
    P = ctypes.c_void_p
    lib.ekf_scalar.argtypes = [P, ctypes.c_int64, P, P, P, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                               ctypes.c_int64, ctypes.c_int64, P]
    x0 = np.array([1.6, 6.0, 0.0, 0.0, np.mean(x)])
    p0 = np.ones(5)
    qd = np.array(kw.get("Q_diag", [1e-8, 1e-8, 1e-6, 1e-6, 1e-8]), dtype=np.float64)
    rv = float(kw["R_val"]) if "R_val" in kw else float(np.var(x))
    out = np.zeros((100, 5))
    lib.ekf_scalar(x.ctypes.data, x.size, x0.ctypes.data, p0.ctypes.data, qd.ctypes.data, rv, 2 * np.pi * e["f_mod"],
                   e["f_samp"], 4000, 100, out.ctypes.data)
    ref = np.stack([d[f"{run}_{k}"] for k in ("amp", "m", "phi", "psi", "dc")], axis=1)
    assert np.abs(out - ref).max() <= 1e-12, np.abs(out - ref).max()
