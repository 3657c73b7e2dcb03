"""CPU pre-validation of the product's fp64 numerics (Bessel walk, per-segment LM)
through a TEST-ONLY host build of the same headers (tests/hostcheck). The GPU
parity tests are the real gate; these catch numerics regressions without a GPU."""
import ctypes
import os

import numpy as np
import pytest

from conftest import check_lm_group, wrapped

HC = os.path.join(os.path.dirname(__file__), "hostcheck", "libhostcheck.so")


@pytest.fixture(scope="module")
def hc():
    if not os.path.exists(HC):
        pytest.skip("hostcheck not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(HC)
    P = ctypes.c_void_p
    lib.hc_bessel_table.argtypes = [ctypes.c_double, ctypes.c_int, P]
    lib.hc_bessel_regs.argtypes = [ctypes.c_double, ctypes.c_int, P]
    lib.hc_fit_segments.argtypes = [P, ctypes.c_long, ctypes.c_int, P, P, P, ctypes.c_int, P, P, P, ctypes.c_int]
    lib.hc_pymod.argtypes = [P, ctypes.c_int64, ctypes.c_double, P]
    return lib


def test_pymod_matches_python_float_modulo(hc):
    """dfmi_pymod (the phi wrap (phi + pi) % (2 pi) - pi, fit.py:357) with the one-fma
    fmod of dfmi_fmod_pos: bit for bit Python's float %, incl. exact multiples, signed
    zeros, values just below/above multiples of 2 pi and the large-|a| library path."""
    rng = np.random.default_rng(7)
    two_pi = 2 * np.pi
    k = rng.integers(-50, 50, 4000).astype(np.float64)
    a = np.concatenate([
        rng.uniform(-100, 100, 20000), rng.uniform(-1e6, 1e6, 5000), rng.normal(0, 1e-12, 2000),
        k * two_pi, np.nextafter(k * two_pi, np.inf), np.nextafter(k * two_pi, -np.inf),
        [0.0, -0.0, 1e-300, -1e-300, 1e-20, -1e-20, 3.141592653589793, -3.141592653589793, 1e15, -1e15, 1e300,
         -1e300, np.inf, -np.inf, np.nan]])
    out = np.empty_like(a)
    hc.hc_pymod(a.ctypes.data, a.size, two_pi, out.ctypes.data)
    want = np.array([float(v) % two_pi for v in a])
    np.testing.assert_array_equal(np.signbit(out), np.signbit(want))
    np.testing.assert_array_equal(out, want)


def test_bessel_vs_scipy_table(hc):
    """Miller two-pass walk vs scipy.special.jv (the reference's Bessel), n <= 64, |x| <= 64."""
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "bessel.npz"))
    n, x, jv = d["n"], d["x"], d["jv"]
    N = int(n.max())
    out = np.zeros(N + 1)
    ours = np.zeros_like(jv)
    for i, xv in enumerate(x):
        hc.hc_bessel_table(float(xv), N, out.ctypes.data)
        ours[:, i] = out
    err = np.abs(ours - jv)
    assert err[:13].max() <= 1e-15          # orders used at ndata = 10
    assert err.max() <= 3e-15               # every order <= 64
    assert (err.max(0) / np.abs(jv).max(0)).max() <= 2e-14


@pytest.mark.parametrize("nb", [14, 18])
def test_bessel_regs_vs_scipy_table(hc, nb):
    """The LM register path's single Miller pass (lm.h bessel_regs) vs scipy.special.jv."""
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "bessel.npz"))
    x, jv = d["x"], d["jv"][:nb]
    out = np.zeros(nb)
    ours = np.zeros_like(jv)
    for i, xv in enumerate(x):
        hc.hc_bessel_regs(float(xv), nb, out.ctypes.data)
        ours[:, i] = out
    assert np.abs(ours - jv).max() <= 1e-15


def _fit(hc, qi, guess, force_general=0):
    n, nd2 = qi.shape
    consts = np.array([100, 1e-9, 1e-9, 1e-3, 5.0, 30.0, 0.5, 0.05, 0.1, 1e-15])
    lams = np.array([0.0, 1e-7, 1e-5, 1e-3, 1e-1, 1.0, 10.0, 100.0])
    qcm = np.ascontiguousarray(qi.T)
    g = np.ascontiguousarray(guess)
    p = np.zeros((n, 4))
    ssq = np.zeros(n)
    st = np.zeros(n, np.int32)
    hc.hc_fit_segments(qcm.ctypes.data, n, nd2 // 2, g.ctypes.data, consts.ctypes.data, lams.ctypes.data, 8,
                       p.ctypes.data, ssq.ctypes.data, st.ctypes.data, force_general)
    return st, p, ssq


@pytest.mark.parametrize("force_general", [0, 1])
@pytest.mark.parametrize("group", ["10", "5", "20", "30", "62", "edge10"])
def test_host_lm_vectors(hc, lm_npz, group, force_general):
    """Both code paths (register path for ndata <= 16, general two-pass path)."""
    qi, g = lm_npz[f"g{group}_qi"], lm_npz[f"g{group}_guess"]
    st, p, ssq = _fit(hc, qi, g, force_general)
    check_lm_group(lm_npz, group, st, p, ssq)


@pytest.mark.parametrize("group", ["10", "20", "30", "62"])
def test_host_wide_lm_vectors(hc, lm_npz, group):
    """The many-harmonic path (lm.h kWideNd, the device's LM from ndata 17) on the golden LM
    vectors, and its one-walk-per-trial form (kWideNdF, lm_wide_fused) bit for bit equal to it."""
    qi, g = lm_npz[f"g{group}_qi"], lm_npz[f"g{group}_guess"]
    split = _fit(hc, qi, g, 3)
    check_lm_group(lm_npz, group, *split)
    fused = _fit(hc, qi, g, 4)
    for x, y in zip(split, fused):
        np.testing.assert_array_equal(x, y)


def test_host_lm_on_reference_qi(hc, records_npz, manifest):
    """LM on the reference's own QI of the config-1 record, chunk size 1, vs the
    reference's _fit_parallel(chunk size 1) outputs: the BASELINE tolerance 1e-9."""
    qi = records_npz["config1_qi"]
    s0 = np.array([records_npz["config1_c1_" + k][0] for k in ("amp", "m", "phi", "psi")])
    g = np.tile(s0, (qi.shape[0], 1))
    g[0] = [1.6, 6.0, 0.0, 0.0]
    st, p, ssq = _fit(hc, qi, g)
    assert (st == records_npz["config1_c1_fitok"]).all()
    for i, k in ((0, "amp"), (1, "m"), (3, "psi")):
        assert np.abs(p[:, i] - records_npz["config1_c1_" + k]).max() <= 1e-9, k
    assert wrapped(p[:, 2] - records_npz["config1_c1_phi"]).max() <= 1e-9


def test_numpy_summation_plan_is_bit_exact(hc):
    """np_sum.h's plan (the device means of the W-DFMI kernels) == np.sum bit for bit,
    across the block, split and 8192-chunk boundaries."""
    hc.hc_np_sum.argtypes = [ctypes.c_void_p, ctypes.c_int]
    hc.hc_np_sum.restype = ctypes.c_double
    rng = np.random.default_rng(0)
    for n in [1, 2, 7, 8, 9, 100, 127, 128, 129, 200, 255, 256, 257, 1000, 3999, 4000, 4001, 5000, 8191, 8192,
              8193, 12345, 16384, 16385, 30001, 400000, 400001]:
        a = rng.standard_normal(n) * 10 ** rng.uniform(-3, 3, n)
        assert hc.hc_np_sum(a.ctypes.data, n) == np.sum(a), n


@pytest.mark.parametrize("group", ["g5", "g10"])
def test_flattened_descent_equals_nested(hc, lm_npz, group):
    """lm.h lm_descend_flat (the SIMT form the kernels run) makes exactly the nested
    _run_lma_fit loop's solves, trials and acceptances: identical bits."""
    qi, g = lm_npz[group + "_qi"], lm_npz[group + "_guess"]
    a = _fit(hc, qi, g, 0)
    b = _fit(hc, qi, g, 2)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


def test_trial_synthesis_restatement_bit_exact(hc):
    """synth.h (dfmi_synth_asd's generator) built for the host, where cos / sin / log
    are numpy's own libm: numpy's legacy RandomState normal stream and whole asd-mode
    trials (amplitude + df noise, arm-length modulation) bit for bit."""
    import deepfmkit_amd as dfm
    from deepfmkit_amd import physics as P
    hc.hc_mt_gauss.argtypes = [ctypes.c_uint32, ctypes.c_int64, ctypes.c_void_p]
    hc.hc_synth_trial.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p]
    for seed in (0, 1, 5, 12345, 2 ** 32 - 1):
        out = np.zeros(3001)
        hc.hc_mt_gauss(seed, 3001, out.ctypes.data)
        np.testing.assert_array_equal(out, np.random.RandomState(seed).normal(size=3001))
    for (m, an, dn, ns, tn, arm) in [(6.0, 1e-4, 0.0, 0.02, 0, 0.0), (8.0, 3e-4, 2e3, 0.02, 3, 0.0),
                                     (6.0, 0.0, 0.0, 0.01, 2, 1e-7), (20.0, 1e-3, 0.0, 0.05, 7, 0.0)]:
        laser = dfm.LaserConfig()
        laser.f_mod = 1000.0
        laser.amp_n, laser.df_n = an, dn
        ifo = dfm.InterferometerConfig()
        ifo.arml_mod_amp = arm
        dfm.set_laser_df_for_effect(laser, ifo, m)
        cfg = dfm.DFMIObject("main_trial", laser, ifo)
        x = np.asarray(P.SignalGenerator().generate(cfg, ns, mode="asd", trial_num=tn)["main"].samples())
        rec = P.synth_trial_fields(cfg, tn)
        out = np.zeros(x.size)
        hc.hc_synth_trial(rec.ctypes.data, x.size, cfg.f_samp, out.ctypes.data)
        np.testing.assert_array_equal(out, x)


def test_trial_synthesis_second_harmonic_waveform_bit_exact(hc):
    """The second-harmonic distortion waveform (waveforms.second_harmonic_distortion,
    reference waveforms.py:4-23) in synth.h, host build vs the numpy generator, main and
    witness (is_dynamic False) channels, incl. distortion_amp = 0 and kwargs omitted."""
    import deepfmkit_amd as dfm
    from deepfmkit_amd import physics as P
    from deepfmkit_amd import waveforms as W
    hc.hc_synth_trial.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p]
    for (m, da, dp, an, tn, kw) in [(6.0, 0.05, 0.3, 1e-4, 0, True), (9.0, 0.0, 0.0, 0.0, 1, True),
                                    (5.0, 0.2, -1.2, 2e-4, 4, True), (7.0, 0.0, 0.0, 1e-4, 2, False)]:
        laser = dfm.LaserConfig()
        laser.amp_n = an
        laser.waveform_func = W.second_harmonic_distortion
        laser.waveform_kwargs = {"distortion_amp": da, "distortion_phase": dp} if kw else {}
        ifo = dfm.InterferometerConfig()
        dfm.set_laser_df_for_effect(laser, ifo, m)
        cfg = dfm.DFMIObject("main_trial", laser, ifo)
        wit_ifo = dfm.InterferometerConfig()
        wit_ifo.meas_arml = 0.15
        wit = dfm.DFMIObject("witness_trial", laser, wit_ifo)
        assert P.device_synth_supported(cfg)
        chans = P.SignalGenerator().generate(cfg, 0.02, mode="asd", trial_num=tn, witness_config=wit)
        for c, key, dyn in ((cfg, "main", True), (wit, "witness", False)):
            x = np.asarray(chans[key].samples())
            rec = P.synth_trial_fields(c, tn, dynamic=dyn)
            assert int(rec["waveform"]) == 1
            out = np.zeros(x.size)
            hc.hc_synth_trial(rec.ctypes.data, x.size, c.f_samp, out.ctypes.data)
            np.testing.assert_array_equal(out, x)
    laser = dfm.LaserConfig()
    laser.waveform_func = lambda tp: np.cos(tp) ** 3  # a user waveform: host generator only
    assert not P.device_synth_supported(dfm.DFMIObject("x", laser, dfm.InterferometerConfig()))


WAVEFORM_CASES = [  # (waveform_func name, kwargs, expected code): reference waveforms.py:4-90
    ("triangle_wave", {}, 2), ("triangle_wave", {"width": 0.3}, 2), ("triangle_wave", {"width": 1.0}, 2),
    ("triangle_wave", {"width": 0}, 2), ("square_wave", {}, 3), ("square_wave", {"duty": 0.25}, 3),
    ("dfm_like_wave", {}, 4), ("dfm_like_wave", {"harmonics": {3: 0.2, 2: -0.05, 5: 0.01}}, 4),
    ("dfm_like_wave", {"harmonics": {}}, 4), ("dfm_wave", {}, 5), ("dfm_wave", {"m": 2.5, "phi": 0.4}, 5),
    ("second_harmonic_distortion", {"distortion_amp": 0.1}, 1),
]


def test_synth_trial_layout(hc):
    from deepfmkit_amd import physics as P
    hc.hc_sizeof_synth_trial.restype = ctypes.c_int64
    assert hc.hc_sizeof_synth_trial() == P.SYNTH_TRIAL_DTYPE.itemsize


@pytest.mark.parametrize("name,kw,code", WAVEFORM_CASES)
def test_synth_waveforms_match_numpy(hc, name, kw, code):
    """synth.h's waveforms (dfmi_synth_asd) built for the host against the package's
    waveforms (the reference's numpy / scipy.signal expressions) on the phase axis of
    a 20 ms record: triangle / square bit for bit (IEEE operations and np.mod only),
    the cosine-based ones to the host libm (bit for bit here as well), and whole asd
    trials through the numpy generator bit for bit."""
    import deepfmkit_amd as dfm
    from deepfmkit_amd import physics as P
    from deepfmkit_amd import waveforms as W
    laser = dfm.LaserConfig()
    laser.psi = 0.37
    laser.amp_n = 1e-4
    laser.waveform_func = getattr(W, name)
    laser.waveform_kwargs = dict(kw)
    ifo = dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    cfg = dfm.DFMIObject("main_trial", laser, ifo)
    assert P.device_synth_supported(cfg)
    rec = P.synth_trial_fields(cfg, 3)
    assert int(rec["waveform"]) == code
    n = int(0.02 * cfg.f_samp)
    t = np.arange(n) / cfg.f_samp
    want = laser.waveform_func(2 * np.pi * laser.f_mod * t + laser.psi, **laser.waveform_kwargs)
    got = np.zeros(n)
    hc.hc_synth_g.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p]
    hc.hc_synth_g(rec.ctypes.data, n, cfg.f_samp, got.ctypes.data)
    np.testing.assert_array_equal(got, want)
    x = np.asarray(P.SignalGenerator().generate(cfg, 0.02, mode="asd", trial_num=3)["main"].samples())
    hc.hc_synth_trial.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p]
    out = np.zeros(x.size)
    hc.hc_synth_trial(rec.ctypes.data, x.size, cfg.f_samp, out.ctypes.data)
    np.testing.assert_array_equal(out, x)


def test_synth_waveform_limits():
    """Waveform arguments the device table cannot hold fall back to the host generator:
    array-valued kwargs, more than 8 dfm_like_wave harmonics, unknown kwargs."""
    import deepfmkit_amd as dfm
    from deepfmkit_amd import physics as P
    from deepfmkit_amd import waveforms as W
    for f, kw in ((W.triangle_wave, {"width": np.full(4, 0.5)}), (W.dfm_like_wave, {"harmonics": {k: 0.01 for k in
                                                                                                 range(2, 12)}}),
                  (W.dfm_wave, {"m": 1.0, "other": 2}), (W.square_wave, {"duty": True})):
        laser = dfm.LaserConfig()
        laser.waveform_func, laser.waveform_kwargs = f, kw
        assert not P.device_synth_supported(dfm.DFMIObject("x", laser, dfm.InterferometerConfig()))


def test_synth_trial_table_equals_per_trial_fields():
    """physics.synth_trial_table (vectorised over trials) == synth_trial_fields per trial,
    every field bit for bit (both waveforms, noise on/off, arm-length modulation)."""
    import deepfmkit_amd as dfm
    from deepfmkit_amd import physics as P
    from deepfmkit_amd import waveforms as W
    cfgs, nums = [], []
    rng = np.random.default_rng(2)
    for i in range(40):
        laser = dfm.LaserConfig()
        laser.amp = 1.0 + rng.normal(0, 0.1)
        laser.psi = rng.uniform(-1, 1)
        laser.amp_n = [0.0, 1e-4][i % 2]
        laser.df_n = [0.0, 3e3][(i // 2) % 2]
        if i % 3 == 0:
            laser.waveform_func = W.second_harmonic_distortion
            laser.waveform_kwargs = {"distortion_amp": rng.uniform(0, 0.1), "distortion_phase": rng.uniform(-1, 1)}
        elif i % 5 == 1:
            laser.waveform_func = W.dfm_like_wave
            laser.waveform_kwargs = {"harmonics": {2: rng.uniform(0, 0.1), 4: rng.uniform(0, 0.1)}}
        elif i % 7 == 2:
            laser.waveform_func = W.triangle_wave
            laser.waveform_kwargs = {"width": rng.uniform(0, 1)}
        ifo = dfm.InterferometerConfig()
        ifo.phi = rng.uniform(0, 6)
        ifo.arml_mod_amp = [0.0, 1e-7][i % 2]
        dfm.set_laser_df_for_effect(laser, ifo, rng.uniform(3, 12))
        cfgs.append(dfm.DFMIObject("main_trial", laser, ifo))
        nums.append(int(rng.integers(0, 10 ** 6)))
    for dyn in (True, False):
        tab = P.synth_trial_table(cfgs, nums, dyn)
        for c, t, row in zip(cfgs, nums, tab):
            one = P.synth_trial_fields(c, t, dyn)
            assert one.tobytes() == row.tobytes()


def test_worker_trials_within_flat_gate(hc):
    """The LM's algebraic shortcuts (block-diagonal J^T J with the psi cross terms taken
    as the zeros they are, closed-form coeffs, LDL^T solve) against the literal general
    path (per-residual Jacobian, pivoting dgesv-style solve) and the oracle (bit-exact
    with the reference's fit.fit) on the QI of the reference's own efficiency trials
    (tests/golden/workers.json): every fitted m within the flat 1e-9 gate of the
    reference, on both paths (host build: exact division)."""
    import json
    import deepfmkit_amd as dfm
    from deepfmkit_amd import physics as P
    from oracle import nls_oracle as O
    G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "workers.json")))
    for t in G["trials"]:
        laser = dfm.LaserConfig()
        laser.f_mod = 1000.0
        laser.amp_n = t["amp_n"]
        ifo = dfm.InterferometerConfig()
        dfm.set_laser_df_for_effect(laser, ifo, t["m_true"])
        cfg = dfm.DFMIObject("main_trial", laser, ifo)
        x = np.asarray(P.SignalGenerator().generate(cfg, t["n_seconds"], mode="asd",
                                                    trial_num=t["trial_num"])["main"].samples())
        R = int(cfg.f_samp / laser.f_mod * int(laser.f_mod * t["n_seconds"]))
        nd = t["ndata"]
        qi = O.demod_buffer(x[:R], nd, 2 * np.pi * laser.f_mod / cfg.f_samp)[:2 * nd]
        g = np.array([1.6, t["m_true"], 0.0, 0.0])
        _, po, _ = O.fit_segment(nd, qi, g)
        assert po[1] == t["m_fit"]  # the oracle is the reference here
        for general in (0, 1):
            _, p, _ = _fit(hc, qi[None, :], g[None, :], general)
            assert abs(p[0, 1] - po[1]) <= 1e-9, (t, general, abs(p[0, 1] - po[1]))


def test_worker_trial_sensitivity_to_qi_ulps():
    """Why the worker trials are gated at max(1e-9, resolution) and not the flat 1e-9
    (tests/test_gpu_workers.py): the reference's own fit (the oracle, bit-exact with
    fit.fit) of the reference's trial inputs, with the QI moved by relative 1e-14 — the
    size of a summation-order difference over R = 4000 samples (numpy's pairwise mean vs
    the GPU's fold + contraction) — moves m by up to 2.9e-9 on trial 6 (amp_n 1e-3: the
    LM stops one step earlier or later), above the flat gate and within the resolution
    bound conftest.resolution_tol; on every trial the spread stays within that bound."""
    import json
    import deepfmkit_amd as dfm
    from deepfmkit_amd import physics as P
    from oracle import nls_oracle as O
    from conftest import resolution_tol
    G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "workers.json")))
    spread = []
    for t in G["trials"]:
        laser = dfm.LaserConfig()
        laser.f_mod = 1000.0
        laser.amp_n = t["amp_n"]
        ifo = dfm.InterferometerConfig()
        dfm.set_laser_df_for_effect(laser, ifo, t["m_true"])
        cfg = dfm.DFMIObject("main_trial", laser, ifo)
        x = np.asarray(P.SignalGenerator().generate(cfg, t["n_seconds"], mode="asd",
                                                    trial_num=t["trial_num"])["main"].samples())
        R = int(cfg.f_samp / laser.f_mod * int(laser.f_mod * t["n_seconds"]))
        nd = t["ndata"]
        qi = O.demod_buffer(x[:R], nd, 2 * np.pi * laser.f_mod / cfg.f_samp)[:2 * nd]
        g = np.array([1.6, t["m_true"], 0.0, 0.0])
        _, po, _ = O.fit_segment(nd, qi, g)
        rng = np.random.default_rng(0)
        d = 0.0
        for _ in range(16):
            _, p2, _ = O.fit_segment(nd, qi * (1.0 + 1e-14 * rng.standard_normal(qi.size)), g)
            d = max(d, abs(p2[1] - po[1]))
        spread.append(d)
        assert d <= resolution_tol(nd, qi, po)[1], (t, d)
    assert spread[6] > 1e-9, spread


def test_bessel_large_argument_vs_scipy(hc):
    """|x| >= 64 (runaway descents): the Hankel expansion of J_0, J_1 + the upward recurrence
    (dfmi_math.h dfmi_bessel_j01_large) in the general path's table and both register-path
    passes, against scipy.special.jv (tests/golden/bessel_large.npz: orders 0..17, |x| up to
    1e4, both signs) — scipy's own error there is ~3.3e-15 (mpmath) — and against a 30-digit
    mpmath evaluation on 40 of the arguments (ours: 4e-17)."""
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "bessel_large.npz"))
    x, jv = d["x"], d["jv"]
    out = np.zeros(18)
    tab = np.zeros((18, x.size))
    for i, xv in enumerate(x):
        hc.hc_bessel_table(float(xv), 17, out.ctypes.data)
        tab[:, i] = out
    assert np.abs(tab - jv).max() <= 1e-14, np.abs(tab - jv).max()
    mp = pytest.importorskip("mpmath")
    mp.mp.dps = 30
    sub = np.arange(0, x.size, x.size // 40)
    ex = np.array([[float(mp.besselj(k, mp.mpf(float(x[i])))) for i in sub] for k in range(18)])
    assert np.abs(tab[:, sub] - ex).max() <= 2e-16, np.abs(tab[:, sub] - ex).max()
    for nb in (14, 18):
        regs = np.zeros((nb, x.size))
        row = np.zeros(nb)
        for i, xv in enumerate(x):
            hc.hc_bessel_regs(float(xv), nb, row.ctypes.data)
            regs[:, i] = row
        assert np.abs(regs - jv[:nb]).max() <= 1e-14, (nb, np.abs(regs - jv[:nb]).max())
        assert np.abs(regs[:, sub] - ex[:nb]).max() <= 2e-16, (nb, np.abs(regs[:, sub] - ex[:nb]).max())
