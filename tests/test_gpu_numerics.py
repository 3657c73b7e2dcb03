"""GPU checks of device numerics that the record tests reach only indirectly.

- scipy.special.jv (the reference's Bessel, fit.py:106-108, 160, 275-276) vs the
  DEVICE Bessel code the fit kernels inline (dfmi_bessel_eval): the general path's
  two-pass Miller walk over n <= 64, |x| <= 64 and both register-path variants, on
  the golden grid (tests/golden/bessel.npz), with the host check's bounds
  (tests/test_host_numerics.py).
- the bin kernels' prefetch setting (bins_prefetch 0 | 4 | 6) is a schedule, not
  arithmetic: rows and record fits are bit-identical across settings on a batch
  large enough that every wave handles several segments (the prefetch path).
- a record on a non-current GPU is fitted on its own device (multi-GPU hosts only).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _bessel(x, nmax, method):
    from deepfmkit_amd import _lib
    lib = _lib.load()
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.zeros((x.size, nmax + 1))
    _lib.check(lib.dfmi_bessel_eval(_lib.ptr(x), x.size, nmax, method, _lib.ptr(out), _lib.DFMI_MEM_HOST, None),
               "dfmi_bessel_eval")
    return out.T


def test_device_bessel_walk_vs_scipy():
    d = np.load(os.path.join(GOLDEN, "bessel.npz"))
    x, jv = d["x"], d["jv"]
    ours = _bessel(x, int(d["n"].max()), 0)
    err = np.abs(ours - jv)
    assert err[:13].max() <= 1e-15          # orders used at ndata = 10
    assert err.max() <= 3e-15               # every order <= 64
    assert (err.max(0) / np.abs(jv).max(0)).max() <= 2e-14


@pytest.mark.parametrize("method,nmax", [(1, 13), (2, 17)])
def test_device_bessel_register_path_vs_scipy(method, nmax):
    d = np.load(os.path.join(GOLDEN, "bessel.npz"))
    x, jv = d["x"], d["jv"][: nmax + 1]
    assert np.abs(_bessel(x, nmax, method) - jv).max() <= 1e-15


def test_bessel_eval_rejects_bad_orders():
    from deepfmkit_amd import _lib
    lib = _lib.load()
    x = np.zeros(4)
    out = np.zeros(4 * 20)
    assert lib.dfmi_bessel_eval(_lib.ptr(x), 4, 14, 1, _lib.ptr(out), _lib.DFMI_MEM_HOST, None) == -1


@pytest.fixture
def restore_prefetch():
    from deepfmkit_amd import _lib
    lib = _lib.load()
    yield lib
    _lib.check(lib.dfmi_set_tuning(b"bins_prefetch", 4), "dfmi_set_tuning")
    _lib.check(lib.dfmi_set_tuning(b"bins_ilv", 0), "dfmi_set_tuning")


@pytest.mark.parametrize("nd", [10, 3, 16])
def test_bins_prefetch_settings_bit_identical(restore_prefetch, nd):
    """The bin kernel's overlap forms — contraction after the fold with 0, 4 or 6 of the
    next segment's chunks prefetched (bins_prefetch), or interleaved block by block with
    the next segment's load groups (bins_ilv) — give the same bits, rows and
    fits, for 1 or 2 harmonic blocks with and without the rows' spare dc slot."""
    import torch
    from deepfmkit_amd import _lib
    from deepfmkit_amd.fitters import nls_records, w0_of
    lib = restore_prefetch
    nseg, R = 20_000, 4000  # > the resident waves: every wave runs several segments
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    t = torch.arange(R, dtype=torch.float64, device="cuda") / 200000.0
    clean = 1.0 + torch.cos(6.0 * torch.cos(2 * np.pi * 1000.0 * t))
    x = (clean.repeat(nseg) + 0.01 * torch.randn(nseg * R, dtype=torch.float64, device="cuda", generator=g))
    qs = lib.dfmi_qi_row_stride(nd)
    st = torch.cuda.current_stream().cuda_stream
    rows, fits = {}, {}
    # ndata 16: the basis leaves no LDS for the second bin set and row ring (64 KB cap): pf4
    settings = {"plain": (0, 0, None), "pf4": (0, 4, "pf4"), "pf6": (0, 6, "pf6"),
                "ilv": (1, 4, "ilv" if nd <= 12 else "pf4")}
    for name, (ilv, pf, token) in settings.items():
        _lib.check(lib.dfmi_set_tuning(b"bins_ilv", ilv), "dfmi_set_tuning")
        _lib.check(lib.dfmi_set_tuning(b"bins_prefetch", pf), "dfmi_set_tuning")
        r = torch.full((nseg, qs), float("nan"), dtype=torch.float64, device="cuda")
        _lib.check(lib.dfmi_demod_rows(x.data_ptr(), nseg, R, R, nd, w0_of(1000.0, 200000.0), 0, r.data_ptr(),
                                       _lib.DFMI_MEM_DEVICE, st), "dfmi_demod_rows")
        rows[name] = r.cpu().numpy()
        kname = lib.dfmi_last_demod_kernel().decode()
        assert token is None or token in kname, (name, kname)
        if nd == 10:
            cols, ok = nls_records(x.reshape(1, -1), 200000.0, 1000.0, R, nseg, nd)  # fused seed + bins + LM
            fits[name] = (cols.cpu().numpy(), ok.cpu().numpy())
            kname = lib.dfmi_last_demod_kernel().decode()
            assert token is None or token in kname, (name, kname)
    for name in settings:
        np.testing.assert_array_equal(rows[name], rows["pf4"])
        if nd == 10:
            np.testing.assert_array_equal(fits[name][0], fits["pf4"][0])
            np.testing.assert_array_equal(fits[name][1], fits["pf4"][1])
    assert lib.dfmi_set_tuning(b"bins_prefetch", 1) == -1  # only 0 | 4 | 6


def test_record_on_non_current_device():
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU")
    from deepfmkit_amd.fitters import nls_records
    R, nseg = 4000, 64
    t = torch.arange(R, dtype=torch.float64) / 200000.0
    x = (1.0 + torch.cos(6.0 * torch.cos(2 * np.pi * 1000.0 * t))).repeat(nseg).reshape(1, -1)
    ref, _ = nls_records(x.to("cuda:0"), 200000.0, 1000.0, R, nseg, 10)
    torch.cuda.set_device(0)
    other, _ = nls_records(x.to("cuda:1"), 200000.0, 1000.0, R, nseg, 10)
    assert other.device.index == 1
    np.testing.assert_array_equal(other.cpu().numpy(), ref.cpu().numpy())


@pytest.fixture
def restore_lm_tuning():
    from deepfmkit_amd import _lib
    lib = _lib.load()
    yield lib
    for k, v in ((b"lm_refill", 0), (b"lm_waves_per_simd", 1), (b"lm_tile_min", 64), (b"lm_phase", 0),
                 (b"lm_pa", 3)):
        _lib.check(lib.dfmi_set_tuning(k, v), "dfmi_set_tuning")


@pytest.mark.parametrize("nrec", [1, 3])
def test_lm_refill_bit_identical(restore_lm_tuning, nrec):
    """The two-phase LM (csrc/lm_phase.h) and the lane-refill LM (csrc/lm_refill.h; tiles of segments per wave, a lane takes the
    tile's next segment when its fit ends) runs every lane through the same solves, trials
    and acceptances as the one-segment-per-lane kernel: same bits, for the record
    pipeline's row layout (incl. tiles that span records, the seeds' dc carry, noisy
    segments that take the m-grid retry) and for dfmi_lm's component-major input."""
    import torch
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import nls_records
    lib = restore_lm_tuning
    nbuf, R, nd = 3001, 4000, 10
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    t = torch.arange(R, dtype=torch.float64, device="cuda") / 200000.0
    recs = []
    for r in range(nrec):
        clean = 1.0 + torch.cos(0.3 * r + (6.0 + r) * torch.cos(2 * np.pi * 1000.0 * t))
        noise = torch.randn(nbuf * R, dtype=torch.float64, device="cuda", generator=g)
        sig = clean.repeat(nbuf) + 0.01 * noise
        sig[7 * R: 9 * R] = 0.8 * noise[7 * R: 9 * R]  # two noise-only buffers: status 1/2 + m-grid retry
        recs.append(sig)
    x = torch.stack(recs).contiguous()
    res = {}
    # (lm_refill, lm_waves_per_simd, lm_tile_min, lm_phase, lm_pa): the one-segment-per-lane
    # kernel, the refill tiles, and the two-phase form (lm_phase.h) with 1 and 3 passes in phase A
    for setting in ((0, 1, 64, 0, 3), (1, 1, 64, 0, 3), (1, 2, 64, 0, 3), (1, 1, 16, 0, 3), (0, 1, 64, 1, 3),
                    (0, 1, 64, 1, 1)):
        for k, v in zip((b"lm_refill", b"lm_waves_per_simd", b"lm_tile_min", b"lm_phase", b"lm_pa"), setting):
            _lib.check(lib.dfmi_set_tuning(k, v), "dfmi_set_tuning")
        cols, ok = nls_records(x, 200000.0, 1000.0, R, nbuf, nd)
        qi = torch.empty((2 * nd, nbuf), dtype=torch.float64, device="cuda")
        dc = torch.empty(nbuf, dtype=torch.float64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        _lib.check(lib.dfmi_demod(x.data_ptr(), nbuf, R, R, nd, 2 * np.pi * 1000.0 / 200000.0, 0, qi.data_ptr(),
                                  dc.data_ptr(), _lib.DFMI_MEM_DEVICE, st), "dfmi_demod")
        gd = torch.tensor([1.0, 6.0, 0.0, 0.0], dtype=torch.float64, device="cuda")
        p = torch.empty((4, nbuf), dtype=torch.float64, device="cuda")
        ssq = torch.empty(nbuf, dtype=torch.float64, device="cuda")
        stt = torch.empty(nbuf, dtype=torch.int32, device="cuda")
        _lib.check(lib.dfmi_lm(qi.data_ptr(), nbuf, nd, gd.data_ptr(), 0, nbuf, F.lm_config(), p.data_ptr(),
                               ssq.data_ptr(), stt.data_ptr(), _lib.DFMI_MEM_DEVICE, st), "dfmi_lm")
        res[setting] = [a.cpu().numpy() for a in (cols, ok, p, ssq, stt)]
    base = res[(0, 1, 64, 0, 3)]
    assert (base[1] != 0).any() and (base[4] != 0).any()  # the retry path ran
    for setting, arrs in res.items():
        for a, b in zip(arrs, base):
            np.testing.assert_array_equal(a, b, err_msg=str(setting))


def test_init_m_with_parallel_is_accepted():
    """Deliberate divergence: the reference raises TypeError for init_m
    together with parallel=True (fitters.py:366 forwards **kwargs still holding init_m
    to _fit_parallel); here the seed's m is taken from init_m, and the result equals the
    oracle's _fit_parallel (chunk size 1) seeded the same way."""
    import deepfmkit_amd as dfm
    from oracle import nls_oracle as O
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 11.0)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("p", laser, ifo, f_samp=200000.0))
    dff.simulate("p", n_seconds=0.2, mode="snr", snr_db=40.0, trial_num=4)
    raw = dff.raws["p"]
    df = dfm.StandardNLSFitter({"n": 20}).fit(raw, parallel=True, init_m=11.0)
    x = np.asarray(raw.samples(), dtype=np.float64)
    ref = O.fit_record_parallel(x, 200000.0, 1000.0, 20, init_m=11.0, n_cores=9)
    assert (df["fitok"].to_numpy() == ref[:, 6]).all()
    assert np.abs(df["m"].to_numpy() - ref[:, 1]).max() <= 1e-9
