"""GPU parity: the HIP path (through the C ABI) against the golden fixtures made
from the reference (tests/golden/make_golden.py) and against the CPU oracle.

Tolerances (fp64), stated in SURVEY.md §8d / BASELINE.md:
  status-0 segments: |d amp|, |d m|, wrapped |d phi|, |d psi| <= 1e-9,
  dc relative <= 1e-13, ssq relative <= 1e-6, status equal on >= 99.9 %.
"""
import numpy as np
import pytest

from conftest import check_lm_group, compare_fit, make_record, record_tol, sha, wrapped

pytestmark = pytest.mark.gpu

FIT_COLS = ("amp", "m", "phi", "psi", "dc", "ssq", "fitok")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from deepfmkit_amd import _lib
    _lib.load()
    assert _lib.load().dfmi_device_count() >= 1


def golden_records(manifest):
    return [e for e in manifest["records"] if e["name"] != "ragged_tail"]


def ref_cols(npz, name, mode):
    return {k: npz[f"{name}_{mode}_{k}"] for k in FIT_COLS}


def df_cols(df):
    return {k: df[k].to_numpy() for k in FIT_COLS}


def test_demod_matches_reference_quadratures(manifest, records_npz):
    """fit.py:18-66 + means: QI and dc of every buffer of every golden record,
    fold kernel (integer period) and direct kernel (non-integer period)."""
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import w0_of
    for e in golden_records(manifest):
        dff = make_record(e)
        x = dff.raws[e["name"]].samples()
        assert sha(x) == e["sha256"], e["name"]
        R, nbuf, nd = e["R"], e["nbuf"], e["ndata"]
        qi, dc = F.demodulate(x[: nbuf * R].reshape(nbuf, R), nd, w0_of(e["f_mod"], e["f_samp"]))
        rqi, rdc = records_npz[f"{e['name']}_qi"], records_npz[f"{e['name']}_dc"]
        assert np.abs(qi - rqi).max() <= 1e-12, (e["name"], np.abs(qi - rqi).max())
        assert (np.abs(dc - rdc) / np.abs(rdc)).max() <= 1e-13, e["name"]


def test_demod_direct_kernel_forced(manifest, records_npz):
    """period=-1 forces the per-sample-sincos kernel on an integer-period record."""
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import w0_of
    e = [r for r in manifest["records"] if r["name"] == "phi1_psi05"][0]
    x = make_record(e).raws[e["name"]].samples()
    R, nbuf, nd = e["R"], e["nbuf"], e["ndata"]
    qi, dc = F.demodulate(x.reshape(nbuf, R), nd, w0_of(e["f_mod"], e["f_samp"]), period=-1)
    assert np.abs(qi - records_npz[f"{e['name']}_qi"]).max() <= 1e-12


@pytest.mark.parametrize("group", ["10", "5", "20", "30", "62", "edge10"])
def test_lm_vectors(lm_npz, group):
    """fit.fit (fit.py:322-361) on (QI, guess) vectors incl. a<0 / m<0 seeds,
    noise up to 0.3, ndata 5..62, all-zero data, a=0 and m=0 seeds."""
    from deepfmkit_amd import fit as F
    qi, g = lm_npz[f"g{group}_qi"], lm_npz[f"g{group}_guess"]
    nd = qi.shape[1] // 2
    st, p, ssq = F.fit_batch(nd, qi, g)
    check_lm_group(lm_npz, group, st, p, ssq)


@pytest.mark.parametrize("mode", ["seq", "c1", "par4"])
def test_records_through_fitter(manifest, records_npz, mode):
    """StandardNLSFitter (fitters.py:330-447) on every golden record:
    seq = _fit_sequential, c1 = _fit_parallel with chunk size 1, par4 = n_cores=4."""
    from deepfmkit_amd.fitters import StandardNLSFitter
    for e in golden_records(manifest):
        key = f"{e['name']}_{mode}_amp"
        if key not in records_npz.files:
            continue
        raw = make_record(e).raws[e["name"]]
        kw = dict(ndata=e["ndata"], init_m=e["init_m"])
        if mode == "seq":
            df = StandardNLSFitter({"n": e["n"]}).fit(raw, parallel=False, **kw)
        elif mode == "c1":
            df = StandardNLSFitter({"n": e["n"]}).fit(raw, parallel=True, **kw)
        else:
            df = StandardNLSFitter({"n": e["n"]}).fit(raw, parallel=True, n_cores=4, **kw)
        ref = ref_cols(records_npz, e["name"], mode)
        # noise-dominated records (SNR <= 0 dB) are status 2 almost everywhere; their
        # status must match, their parameters are reported, not gated.
        # Status-0 segments: 1e-9, widened only where the reference's own ssq resolution
        # is coarser (record_tol: the SNR 0 dB record's status-0 segments, ssq ~1e-3)
        tol = record_tol(e["ndata"], records_npz[f"{e['name']}_qi"], ref)
        compare_fit(df_cols(df), ref, tol=tol)


def test_facade_tau_and_time(manifest, records_npz):
    """DeepFitFramework.fit (core.py:424-517): tau = m/(2 pi df), time axis."""
    e = [r for r in manifest["records"] if r["name"] == "config1"][0]
    dff = make_record(e)
    fobj = dff.fit(e["name"], n=e["n"], parallel=False, ndata=e["ndata"])
    np.testing.assert_allclose(fobj.tau, records_npz["config1_facade_tau"], rtol=0, atol=1e-18)
    np.testing.assert_array_equal(fobj.time, records_npz["config1_facade_time"])
    assert (fobj.R, fobj.nbuf, fobj.n) == (e["facade"]["R"], e["facade"]["nbuf"], e["facade"]["n"])


def test_asd_two_channel_batch():
    """Config 3 (notebooks/0.1_quickstart-2-ch): main m=6 + witness m=4.3, asd mode,
    fitted as ONE batch of 2 records (fit_many) and one by one."""
    import os
    import deepfmkit_amd as dfm
    from deepfmkit_amd.data import DeepRawObject
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "asd_pair.npz"))
    dff = dfm.DeepFitFramework()
    for key in ("dynamic_channel", "reference_channel"):
        raw = DeepRawObject(data=d[f"{key}_x"])
        raw.label, raw.f_samp, raw.f_mod, raw.t0 = key, 200000.0, 1000, 0
        dff.raws[key] = raw
    out = dff.fit_many(["dynamic_channel", "reference_channel"], n=20, parallel=False)
    for key in ("dynamic_channel", "reference_channel"):
        fo = out[key]
        ours = dict(amp=fo.amp, m=fo.m, phi=fo.phi, psi=fo.psi, dc=fo.dc, ssq=fo.ssq,
                    fitok=dff.fits_df[f"{key}_nls"]["fitok"].to_numpy())
        ref = {k: d[f"{key}_{k}"] for k in FIT_COLS}
        compare_fit(ours, ref, tol=1e-9)


def test_ekf_matches_reference(manifest):
    """EKFFitter (fitters.py:214-320) snapshot states, default and tuned Q/R."""
    import os
    import deepfmkit_amd as dfm
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "ekf.npz"))
    e = manifest["ekf"]
    dff = make_record(e)
    x = dff.raws["ekf"].samples()
    assert sha(x) == e["sha256"]
    dff.fit("ekf", method="ekf", fit_label="d", n=20)
    dff.fit("ekf", method="ekf", fit_label="t", n=20, Q_diag=[1e-9, 1e-9, 1e-7, 1e-7, 1e-9], R_val=0.001)
    for lab, ref in (("d", "ekf_default"), ("t", "ekf_tuned")):
        df = dff.fits_df[lab]
        for k in ("amp", "m", "phi", "psi", "dc"):
            err = np.abs(df[k].to_numpy() - d[f"{ref}_{k}"]).max()
            assert err <= 1e-9, (lab, k, err)


# EKF kernels: (ekf_row, ekf_rot) tuning and the kernel dfmi_last_demod_kernel reports.
# rot: 16-lane row per channel, sincos by rotation between anchors (default for few
# channels, R % 4 == 0); row: the same row with the full sincos per sample; lanerot / lane:
# one lane per channel (many channels) with / without the rotation.
# pit: parallel in time (ekf_pit.h), the default for up to 1024 channels of >= 4096 samples;
# here forced on from 1024 samples so the shorter records take it too.
EKF_KERNELS = {"rot": (1, 1, "ekf_rot_kernel"), "row": (1, 0, "ekf_row_kernel"), "lanerot": (0, 1, "ekf_lane_rot_kernel"),
               "lane": (0, 0, "ekf_kernel"), "pit": (1, 1, "ekf_pit")}


class _ekf_kernel:
    """Selects one EKF kernel by tuning; kname: the prefix dfmi_last_demod_kernel reports."""

    def __init__(self, lib, name):
        self.lib, self.row, self.rot, self.kname = lib, *EKF_KERNELS[name]
        self.pit = name == "pit"

    def __enter__(self):
        from deepfmkit_amd import _lib
        _lib.check(self.lib.dfmi_set_tuning(b"ekf_row", self.row), "tune")
        _lib.check(self.lib.dfmi_set_tuning(b"ekf_rot", self.rot), "tune")
        _lib.check(self.lib.dfmi_set_tuning(b"ekf_pit", 1024 if self.pit else 0), "tune")
        _lib.check(self.lib.dfmi_set_tuning(b"ekf_pit_min", 1024 if self.pit else 4096), "tune")
        return self

    def __exit__(self, *exc):
        from deepfmkit_amd import _lib
        for key, v in ((b"ekf_row", 1), (b"ekf_rot", 1), (b"ekf_pit", 1024), (b"ekf_pit_min", 4096)):
            _lib.check(self.lib.dfmi_set_tuning(key, v), "tune")

    def used(self):
        return self.lib.dfmi_last_demod_kernel().decode().startswith(self.kname)


def _c_ekf(x, init4, R, nbuf, f_samp=200000.0, f_mod=1000.0, qd=(1e-8, 1e-8, 1e-6, 1e-6, 1e-8)):
    """The oracle's scalar C restatement of EKFFitter.fit (oracle/csrc/ekf_scalar.c, pinned to
    the numpy oracle by tests/test_oracle_c.py) on one record; None when not built."""
    import ctypes
    import os
    so = os.path.join(os.path.dirname(os.path.dirname(__file__)), "oracle", "libekf_scalar.so")
    if not os.path.exists(so):
        return None
    cl = ctypes.CDLL(so)
    P = ctypes.c_void_p
    cl.ekf_scalar.argtypes = [P, ctypes.c_int64, P, P, P, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                              ctypes.c_int64, ctypes.c_int64, P]
    x = np.ascontiguousarray(x, dtype=np.float64)
    x0 = np.array(list(init4) + [np.mean(x)])
    p0, q = np.ones(5), np.ascontiguousarray(qd, dtype=np.float64)
    ref = np.zeros((nbuf, 5))
    cl.ekf_scalar(x.ctypes.data, x.size, x0.ctypes.data, p0.ctypes.data, q.ctypes.data, float(np.var(x)),
                  2 * np.pi * f_mod, f_samp, R, nbuf, ref.ctypes.data)
    return ref


@pytest.mark.parametrize("kern", ["rot", "row", "lanerot", "lane", "pit"])
def test_ekf_long_record_matches_oracle(kern):
    """Config 5 shape on a longer record than the golden one (0.1 s = 20,000 samples,
    5 snapshots): every EKF kernel — one 16-lane row per channel with sincos by rotation
    (ekf_rot_kernel, the default for few channels) or in full per sample (ekf_row_kernel),
    one lane per channel (ekf_kernel) — tracks the restated reference loop to fp64 rounding
    (the reference itself moves by ~1e-15 under 1-ulp input changes), and several channels in
    one launch give each channel's answer bit for bit."""
    import deepfmkit_amd as dfm
    from deepfmkit_amd import _lib
    from oracle import nls_oracle as O
    lib = _lib.load()
    with _ekf_kernel(lib, kern) as k:
        _ekf_long_record(dfm, O, lib, k)


def _ekf_long_record(dfm, O, lib, kk):
    laser = dfm.LaserConfig()
    ifo = dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("e", laser, ifo, f_samp=200000.0))
    dff.simulate("e", n_seconds=0.1, mode="snr", snr_db=40.0, trial_num=5)
    raw = dff.raws["e"]
    x = np.asarray(raw.samples(), dtype=np.float64)
    ref = O.ekf_record(x, 200000.0, 1000.0, 20)
    got = dfm.fitters.ekf_records([raw], 20)[0]
    assert kk.used(), lib.dfmi_last_demod_kernel()
    assert np.max(np.abs(got - ref)) <= 1e-12, np.max(np.abs(got - ref))
    # row kernel: a second wave, rows past the end; parallel in time: 20,000 samples give the
    # minimum block (16) for 1 and for 6 channels alike, so the runs are bit-comparable
    many = dfm.fitters.ekf_records([raw] * 6, 20)
    for k in range(6):
        np.testing.assert_array_equal(many[k], got)


@pytest.mark.parametrize("kern", ["rot", "row", "lanerot", "lane", "pit"])
def test_ekf_config5_full_length_matches_c_oracle(kern):
    """Config 5 at the length BASELINE names (notebooks/2.0 defaults):
    a 2 s = 400,000-sample snr-mode record (m=6, 40 dB) through dfmi_ekf_fit (EKFFitter.fit,
    fitters.py:214-320, pre-reductions on the device) with every EKF kernel, against the
    oracle's scalar C restatement of the loop (oracle/csrc/ekf_scalar.c, pinned to the
    numpy oracle by tests/test_oracle_c.py) on every one of the 100 snapshots."""
    import deepfmkit_amd as dfm
    from deepfmkit_amd import _lib
    lib = _lib.load()
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("c5", laser, ifo, f_samp=200000.0))
    dff.simulate("c5", n_seconds=2.0, mode="snr", snr_db=40.0, trial_num=7)
    raw = dff.raws["c5"]
    x = np.ascontiguousarray(raw.samples(), dtype=np.float64)
    assert x.size == 400_000
    ref = _c_ekf(x, [1.6, 6.0, 0.0, 0.0], 4000, 100)
    if ref is None:
        pytest.skip("oracle/libekf_scalar.so not built (make -C oracle)")
    with _ekf_kernel(lib, kern) as k:
        got = dfm.fitters.ekf_records([raw], 20)[0]
        assert k.used(), lib.dfmi_last_demod_kernel()
    assert got.shape == (100, 5)
    err = np.abs(got - ref)
    assert err.max() <= 1e-12, (err.max(), np.unravel_index(err.argmax(), err.shape))
    assert abs(got[-1, 1] - 6.0) < 1e-2  # the filter tracks m


def _ekf_raw(dfm, m, f_samp, f_mod, seconds, trial):
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    laser.f_mod = f_mod
    dfm.set_laser_df_for_effect(laser, ifo, m)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("r", laser, ifo, f_samp=f_samp))
    dff.simulate("r", n_seconds=seconds, mode="snr", snr_db=40.0, trial_num=trial)
    return dff.raws["r"]


@pytest.mark.parametrize("kern", ["rot", "lanerot"])
@pytest.mark.parametrize("m,f_samp,f_mod", [(25.0, 32000.0, 400.0), (10.0, 32000.0, 400.0),
                                            (10.0, 32160.0, 400.0), (6.0, 30000.0, 400.0)])
def test_ekf_rotation_fallback_groups_match_c_oracle(m, f_samp, f_mod, kern):
    """ekf_rot_kernel / ekf_lane_rot_kernel where the phase argument moves by more than the rotation's 0.78 rad per
    sample (m = 25 / 10 at 400 Hz, 32 kS/s: up to 1.96 / 0.79 rad): those groups are rolled
    back and re-run with the full sincos, the rest rotate; R = 1600 (groups of 16), 1608 (of 8)
    and 1500 (of 4). States within 1e-12 of the scalar C restatement on every snapshot, init_m
    at the true m."""
    import deepfmkit_amd as dfm
    from deepfmkit_amd import _lib
    lib = _lib.load()
    raw = _ekf_raw(dfm, m, f_samp, f_mod, 1.0, 3)
    x = np.ascontiguousarray(raw.samples(), dtype=np.float64)
    R = int(round(f_samp / f_mod * 20))
    nbuf = x.size // R
    ref = _c_ekf(x, [1.6, m, 0.0, 0.0], R, nbuf, f_samp, f_mod)
    if ref is None:
        pytest.skip("oracle/libekf_scalar.so not built (make -C oracle)")
    with _ekf_kernel(lib, kern) as k:
        got = dfm.fitters.ekf_records([raw], 20, init_m=m)[0]
        assert k.used(), lib.dfmi_last_demod_kernel()
    err = np.abs(got - ref)
    assert err.max() <= 1e-12, (err.max(), np.unravel_index(err.argmax(), err.shape))


@pytest.mark.parametrize("kern", ["rot", "lanerot"])
def test_ekf_rotation_channels_independent_and_ragged_tail(kern):
    """A channel's ekf_rot_kernel / ekf_lane_rot_kernel result never depends on the other channels of its wave:
    channels that take the fallback (m = 25) and channels that rotate (m = 2) in one launch
    equal their single-channel runs bit for bit; a record whose length is not a multiple of
    the group (20,003 samples) fits its tail samples with the full sincos and matches the
    numpy oracle within 1e-12; R % 4 != 0 selects ekf_row_kernel."""
    import deepfmkit_amd as dfm
    from deepfmkit_amd import _lib
    from oracle import nls_oracle as O
    lib = _lib.load()
    ra = _ekf_raw(dfm, 25.0, 32000.0, 400.0, 0.5, 1)
    rb = _ekf_raw(dfm, 2.0, 32000.0, 400.0, 0.5, 2)
    with _ekf_kernel(lib, kern) as kk:
        a = dfm.fitters.ekf_records([ra], 20, init_m=6.0)[0]
        b = dfm.fitters.ekf_records([rb], 20, init_m=6.0)[0]
        mix = dfm.fitters.ekf_records([ra, rb, rb, ra, rb], 20, init_m=6.0)
        assert kk.used(), lib.dfmi_last_demod_kernel()
        for k, want in enumerate((a, b, b, a, b)):
            np.testing.assert_array_equal(mix[k], want)
        # ragged tail: 20,003 samples, R = 4000
        dff = dfm.DeepFitFramework()
        laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
        dfm.set_laser_df_for_effect(laser, ifo, 6.0)
        dff.load_sim(dfm.DFMIObject("t", laser, ifo, f_samp=200000.0))
        dff.simulate("t", n_seconds=0.1, mode="snr", snr_db=40.0, trial_num=4)
        raw = dff.raws["t"]
        x = np.asarray(raw.samples(), dtype=np.float64)
        x = np.concatenate([x, x[:3]])
        got = _ekf_host(lib, x, 200000.0, 1000.0, 4000, 5)
        assert kk.used(), lib.dfmi_last_demod_kernel()
        ref = O.ekf_record(x, 200000.0, 1000.0, 20)
        assert np.max(np.abs(got - ref)) <= 1e-12
        # an odd R (1501 samples per snapshot): no group can end on the snapshots -> no rotation
        _ekf_host(lib, x[:6 * 1501], 30020.0, 400.0, 1501, 6)
        assert lib.dfmi_last_demod_kernel().decode() == ("ekf_row_kernel" if kern == "rot" else "ekf_kernel")


def _ekf_host(lib, x, f_samp, f_mod, R, nbuf):
    from deepfmkit_amd import _lib
    x = np.ascontiguousarray(x, dtype=np.float64)
    init4 = np.array([1.6, 6.0, 0.0, 0.0])
    p0, qd = np.ones(5), np.array([1e-8, 1e-8, 1e-6, 1e-6, 1e-8])
    states = np.zeros((1, nbuf, 5))
    _lib.check(lib.dfmi_ekf_fit(_lib.ptr(x), 1, x.size, x.size, _lib.ptr(init4), _lib.ptr(p0), _lib.ptr(qd), None,
                                2 * np.pi * f_mod, f_samp, R, nbuf, _lib.ptr(states), _lib.DFMI_MEM_HOST, None),
               "dfmi_ekf_fit")
    return states[0]


@pytest.mark.parametrize("n", [1, 7, 8, 127, 129, 4000, 8191, 8192, 8193, 30001, 400000, 800000])
def test_record_moments_bit_exact(n):
    """dfmi_record_moments == np.mean / np.var bit for bit (numpy's pairwise tree, its
    8192-element buffer chunks, (x - mean)^2 rounded per operation), for 3 strided
    records, from host and from device memory; 800,000 samples take the tree kernel's
    global-memory node path (more nodes than its LDS holds)."""
    import torch
    from deepfmkit_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(n)
    stride = n + 5
    x = rng.standard_normal(3 * stride) * 10 ** rng.uniform(-2, 2, 3 * stride) + 1.7
    mean, var = np.zeros(3), np.zeros(3)
    _lib.check(lib.dfmi_record_moments(_lib.ptr(x), 3, stride, n, _lib.ptr(mean), _lib.ptr(var),
                                       _lib.DFMI_MEM_HOST, None), "dfmi_record_moments")
    for r in range(3):
        xr = x[r * stride: r * stride + n]
        assert mean[r] == np.mean(xr), (n, r)
        assert var[r] == np.var(xr), (n, r)
    dx = torch.from_numpy(x).cuda()
    dm, dv = torch.zeros(3, dtype=torch.float64, device="cuda"), torch.zeros(3, dtype=torch.float64, device="cuda")
    st = torch.cuda.current_stream()
    _lib.check(lib.dfmi_record_moments(dx.data_ptr(), 3, stride, n, dm.data_ptr(), dv.data_ptr(),
                                       _lib.DFMI_MEM_DEVICE, st.cuda_stream), "dfmi_record_moments")
    np.testing.assert_array_equal(dm.cpu().numpy(), mean)
    np.testing.assert_array_equal(dv.cpu().numpy(), var)


@pytest.mark.parametrize("r_val", [None, 0.001])
def test_ekf_device_prereductions_equal_host_numpy(r_val):
    """dfmi_ekf_fit (np.mean / np.var on the device, fitters.py:253, 256) == dfmi_ekf
    handed numpy's own mean and variance: the same states, bit for bit."""
    import deepfmkit_amd as dfm
    from deepfmkit_amd import _lib
    lib = _lib.load()
    laser = dfm.LaserConfig()
    ifo = dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("e", laser, ifo, f_samp=200000.0))
    dff.simulate("e", n_seconds=0.1, mode="snr", snr_db=40.0, trial_num=3)
    raw = dff.raws["e"]
    x = np.ascontiguousarray(raw.samples(), dtype=np.float64)
    got = dfm.fitters.ekf_records([raw], 20, **({} if r_val is None else {"R_val": r_val}))[0]
    x0 = np.array([1.6, 6.0, 0.0, 0.0, np.mean(x)])
    rv = np.array([np.var(x) if r_val is None else r_val])
    p0 = np.ones(5)
    qd = np.array([1e-8, 1e-8, 1e-6, 1e-6, 1e-8])
    nbuf = x.size // 4000
    ref = np.zeros((nbuf, 5))
    _lib.check(lib.dfmi_ekf(_lib.ptr(x), 1, x.size, x.size, _lib.ptr(x0), _lib.ptr(p0), _lib.ptr(qd), _lib.ptr(rv),
                            2 * np.pi * 1000.0, 200000.0, 4000, nbuf, _lib.ptr(ref), _lib.DFMI_MEM_HOST, None),
               "dfmi_ekf")
    np.testing.assert_array_equal(got, ref)


def test_large_batch_known_answer_and_seed_independence():
    """Full-size property checks (config 2 shape, 100k segments of R=4000, on device):
    noiseless A(1+cos(phi+m cos(wt+psi))) is recovered exactly in every segment, and a
    segment's result does not depend on the batch it is fitted in (chunk size 1)."""
    import torch
    from deepfmkit_amd.fitters import nls_records
    nseg, R = 100_000, 4000
    t = torch.arange(R, dtype=torch.float64, device="cuda") / 200000.0
    seg_phi = torch.linspace(-0.5, 0.5, nseg, dtype=torch.float64, device="cuda")
    w = 2 * np.pi * 1000.0
    x = (1.0 + torch.cos(seg_phi[:, None] + 6.0 * torch.cos(w * t[None, :] + 0.1))).reshape(1, -1)
    cols, ok = nls_records(x, 200000.0, 1000.0, R, nseg, 10)
    cols = cols.cpu().numpy()
    ok = ok.cpu().numpy()
    assert (ok == 0).all()
    assert np.abs(cols[0] - 1.0).max() < 1e-9
    assert np.abs(cols[1] - 6.0).max() < 1e-9
    assert wrapped(cols[2] - seg_phi.cpu().numpy()).max() < 1e-9
    assert np.abs(cols[3] - 0.1).max() < 1e-9
    # seed independence: refit a slice alone, seeded identically (segment 0 of the big batch)
    sub = x[:, 5000 * R: 5100 * R].contiguous()
    sub_all = torch.cat([x[:, :R], sub], dim=1)
    cols2, _ = nls_records(sub_all, 200000.0, 1000.0, R, 101, 10)
    np.testing.assert_array_equal(cols2.cpu().numpy()[:, 1:], cols[:, 5000:5100])


def _demod_both(x, nseg, R, nd, w0):
    """dfmi_demod (component-major) and dfmi_demod_rows (record-pipeline rows) on device data."""
    import torch
    from deepfmkit_amd import _lib
    lib = _lib.load()
    st = torch.cuda.current_stream().cuda_stream
    qi = torch.empty((2 * nd, nseg), dtype=torch.float64, device="cuda")
    dc = torch.empty(nseg, dtype=torch.float64, device="cuda")
    _lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0, 0, qi.data_ptr(), dc.data_ptr(),
                              _lib.DFMI_MEM_DEVICE, st), "dfmi_demod")
    qs = lib.dfmi_qi_row_stride(nd)
    rows = torch.full((nseg, qs), float("nan"), dtype=torch.float64, device="cuda")
    _lib.check(lib.dfmi_demod_rows(x.data_ptr(), nseg, R, R, nd, w0, 0, rows.data_ptr(), _lib.DFMI_MEM_DEVICE, st),
               "dfmi_demod_rows")
    torch.cuda.synchronize()
    return qi.cpu().numpy(), dc.cpu().numpy(), rows.cpu().numpy(), qs, lib.dfmi_qi_row_dc(nd)


@pytest.mark.parametrize("nd", [10, 3, 8, 16])
def test_demod_rows_bit_identical_to_component_major(nd):
    """The record pipeline's row layout (full-line stores, dc inside the row) carries
    exactly the values of dfmi_demod's bin kernel; unused slots are 0. ndata 8/16 have no
    spare slot (dc in an 8-double tail). (From 13 harmonics dfmi_demod runs
    demod_wide_kernel by default, tests/test_gpu_demod_wide.py; demod_wide = 0 here.)"""
    import torch
    from deepfmkit_amd import _lib
    from deepfmkit_amd.fitters import w0_of
    lib = _lib.load()
    nseg, R = 3001, 4000
    g = torch.Generator(device="cuda")
    g.manual_seed(nd)
    x = torch.randn(nseg * R, dtype=torch.float64, device="cuda", generator=g) + 0.25
    _lib.check(lib.dfmi_set_tuning(b"demod_wide", 0), "tune")
    try:
        qi, dc, rows, qs, dpos = _demod_both(x, nseg, R, nd, w0_of(1000.0, 200000.0))
    finally:
        _lib.check(lib.dfmi_set_tuning(b"demod_wide", 1), "tune")
    nblk = (nd + 7) // 8
    assert qs == 16 * nblk + (0 if nd % 8 else 8)
    used = np.zeros(qs, bool)
    for h in range(nd):
        b, i = divmod(h, 8)
        np.testing.assert_array_equal(rows[:, 16 * b + i], qi[h])
        np.testing.assert_array_equal(rows[:, 16 * b + 8 + i], qi[nd + h])
        used[16 * b + i] = used[16 * b + 8 + i] = True
    np.testing.assert_array_equal(rows[:, dpos], dc)
    used[dpos] = True
    written = np.arange(qs) < 16 * nblk
    assert (rows[:, ~used & written] == 0).all()


def test_record_rows_path_matches_component_path():
    """dfmi_nls_record through the row layout (default for chunk size 1) is
    bit-identical to the component-major path (forced with demod_kernel = 0), for a
    multi-record strided batch and for nbuf = 1 (the dc of the seed buffers): the seed
    of both paths is the LDS bin fold of buffer 0 (seed_bins_kernel)."""
    import torch
    from deepfmkit_amd import _lib
    from deepfmkit_amd.fitters import nls_records
    lib = _lib.load()
    R = 4000
    t = torch.arange(40 * R, dtype=torch.float64, device="cuda") / 200000.0
    w = 2 * np.pi * 1000.0
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    base = torch.stack([1.0 + torch.cos(0.3 * k + (5.5 + 0.2 * k) * torch.cos(w * t + 0.1 * k)) for k in range(3)])
    recs = torch.zeros((3, 41 * R), dtype=torch.float64, device="cuda")  # rec_stride > nbuf * R
    recs[:, : 40 * R] = base + 1e-3 * torch.randn(base.shape, dtype=torch.float64, device="cuda", generator=g)
    for nbuf in (40, 1):
        res = {}
        for kern in (1, 0):
            _lib.check(lib.dfmi_set_tuning(b"demod_kernel", kern), "tune")
            cols, ok = nls_records(recs, 200000.0, 1000.0, R, nbuf, 10)
            res[kern] = (cols.cpu().numpy(), ok.cpu().numpy(), lib.dfmi_last_demod_kernel().decode())
        _lib.check(lib.dfmi_set_tuning(b"demod_kernel", 1), "tune")
        a, b = res[1], res[0]
        assert "rows" in a[2] and "rows" not in b[2], (a[2], b[2])
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])


@pytest.mark.parametrize("nrec,nbuf", [(3, 40), (600, 3), (4, 1), (1, 2), (1, 300)])
def test_fused_seed_layouts_match_unfused(nrec, nbuf):
    """The fused seed + demodulation launch (contiguous records) against the two-kernel
    path (the same records laid out with rec_stride > nbuf*R: seed kernel on the side
    stream beside the bulk demodulation) across layouts: several records (one seed
    workgroup each), more records than can be resident as seeds (the fused path steps
    aside), single-buffer records (no LM), two buffers. Same bits; every record's seed
    is its own buffer 0 (fitters.py:403-410)."""
    import torch
    from deepfmkit_amd import _lib
    from deepfmkit_amd.fitters import nls_records
    lib = _lib.load()
    R = 4000
    t = torch.arange(nbuf * R, dtype=torch.float64, device="cuda") / 200000.0
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    ms = torch.linspace(4.0, 8.0, nrec, dtype=torch.float64, device="cuda")[:, None]
    x = 1.0 + torch.cos(0.3 + ms * torch.cos(2 * np.pi * 1000.0 * t[None, :] + 0.1))
    x = (x + 1e-3 * torch.randn(x.shape, dtype=torch.float64, device="cuda", generator=g)).contiguous()
    # unfused: every record twice (so even nrec = 1 is a multi-record batch), strided
    strided = torch.zeros((2 * nrec, nbuf * R + 2 * R), dtype=torch.float64, device="cuda")
    strided[:nrec, : nbuf * R] = x
    strided[nrec:, : nbuf * R] = x
    res = []
    for arr in (x, strided):
        cols, ok = nls_records(arr, 200000.0, 1000.0, R, nbuf, 10, init_guess=(1.0, 6.0, 0.0, 0.0))
        res.append((cols.cpu().numpy()[:, : nrec * nbuf], ok.cpu().numpy()[: nrec * nbuf],
                    lib.dfmi_last_demod_kernel().decode()))
        if arr is strided:
            np.testing.assert_array_equal(cols.cpu().numpy()[:, nrec * nbuf:], res[-1][0])
    if nrec * 2 < 400 and nbuf > 1:
        assert res[0][2].startswith("demod_seed_bins_kernel"), res[0][2]
    assert not res[1][2].startswith("demod_seed_bins_kernel"), res[1][2]
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])
    m = res[0][0][1].reshape(nrec, nbuf)
    assert np.all(np.abs(m - ms.cpu().numpy()) < 1e-3)
    assert np.all(res[0][1] == 0)


def test_raw_file_to_fit_file_end_to_end(tmp_path):
    """raw_data file -> load_raw (host, and straight to the GPU) -> fit -> to_txt ->
    load_fit: the device-loaded record fits to the same bits as the host-loaded one,
    and the fit file reads back bit-exact."""
    import deepfmkit_amd as dfm
    from deepfmkit_amd import textio
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    src = dfm.DeepFitFramework()
    src.load_sim(dfm.DFMIObject("s", laser, ifo, f_samp=200000.0))
    src.simulate("s", n_seconds=0.1, mode="snr", snr_db=40.0, trial_num=3)
    raw_path = str(tmp_path / "raw_data.txt")
    textio.write_raw(raw_path, [src.raws["s"].samples()], t0=20250101, f_samp=200000.0, f_mod=1000.0)
    fits = {}
    for dev in (None, "cuda:0"):
        dff = dfm.DeepFitFramework()
        dff.load_raw(raw_path, labels=["ch"], device=dev)
        fo = dff.fit("ch", n=20)
        fits[dev] = fo
    for k in ("amp", "m", "phi", "psi", "dc", "ssq"):
        np.testing.assert_array_equal(np.asarray(getattr(fits[None], k)), np.asarray(getattr(fits["cuda:0"], k)))
    fit_path = str(tmp_path / "fit_data.txt")
    fits[None].to_txt(fit_path)
    back = dfm.DeepFitFramework()
    back.raw_file = "x"
    back.load_fit(fit_path)
    fb = back.fits["x_ch0"]
    for k in ("amp", "m", "phi", "psi", "dc", "ssq"):
        assert np.asarray(getattr(fb, k)).tobytes() == np.asarray(getattr(fits[None], k), dtype=np.float64).tobytes()


@pytest.mark.parametrize("kern", ["rot", "row", "lanerot", "lane", "pit"])
@pytest.mark.parametrize("run", ["c5_default", "c5_tuned"])
def test_ekf_config5_full_length_vs_reference(manifest, kern, run):
    """Config 5 at full length against the REFERENCE's own EKFFitter states (2 s = 400,000
    samples, tests/golden/make_ekf_full_golden.py: the defaults of fitters.py:241-257, and a
    second record with tuned Q / R), through DeepFitFramework.fit(method='ekf') with every
    EKF kernel: 1e-9 on all 100 snapshots of amp, m, phi, psi, dc."""
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "ekf_full.npz"))
    e = {r["name"]: r for r in manifest["ekf_full"]}[run]
    dff = make_record(e)
    assert sha(dff.raws[run].samples()) == e["sha256"]
    from deepfmkit_amd import _lib
    lib = _lib.load()
    with _ekf_kernel(lib, kern) as k:
        dff.fit(run, method="ekf", fit_label="f", n=20, **e["fit_kwargs"])
        assert k.used(), lib.dfmi_last_demod_kernel()
    df = dff.fits_df["f"]
    assert len(df) == 100
    for c in ("amp", "m", "phi", "psi", "dc"):
        err = np.abs(df[c].to_numpy() - d[f"{run}_{c}"]).max()
        assert err <= 1e-9, (c, err)
