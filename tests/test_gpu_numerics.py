"""GPU checks of device numerics that the record tests reach only indirectly.

- scipy.special.jv (the reference's Bessel, fit.py:106-108, 160, 275-276) vs the
  DEVICE Bessel code the fit kernels inline (dfmi_bessel_eval): the general path's
  two-pass Miller walk over n <= 64, |x| <= 64 and both register-path variants, on
  the golden grid (tests/golden/bessel.npz), with the host check's bounds
  (tests/test_host_numerics.py).
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
def restore_ladder():
    from deepfmkit_amd import _lib
    lib = _lib.load()
    yield lib
    _lib.check(lib.dfmi_set_tuning(b"lm_ladder", 32), "dfmi_set_tuning")
    _lib.check(lib.dfmi_set_tuning(b"lm_ladder_split", 4), "dfmi_set_tuning")


@pytest.mark.parametrize("nd", [10, 7, 30])
def test_lm_ladder_bit_identical(restore_ladder, nd):
    """The parallel lambda ladder (lm.h lm_descend_ladder: 8 lanes per segment, every
    rung of an LM iteration tried in one pass, the first improving one taken) accepts
    exactly the points of the one-lane descent: same bits for the warm-start chains of
    _fit_sequential and of n_cores chunks, for a small chunk-size-1 record (row layout),
    and for dfmi_lm's per-segment guesses — incl. noise-only buffers that take the m-grid
    retry (status 1/2), the register path (ndata 10 exact, 7 masked) and the general
    path (ndata 30). Beyond 16 harmonics the ladder's small batches default to one wave per
    segment, 8 rungs x 8 harmonic shares (lm_ladder_split): sums in another order, so that form
    is held to the one-lane descent's status and, on status-0 fits, to 1e-7 (its parity against
    the reference: tests/test_gpu_quickstart.py), and the bit identity to lm_ladder_split 0."""
    import torch
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import nls_records
    lib = restore_ladder
    nbuf, R, nrec = 301, 4000, 3
    g = torch.Generator(device="cuda")
    g.manual_seed(5 + nd)
    t = torch.arange(R, dtype=torch.float64, device="cuda") / 200000.0
    recs = []
    for r in range(nrec):
        clean = 1.0 + torch.cos(0.3 * r + (6.0 + r) * torch.cos(2 * np.pi * 1000.0 * t))
        noise = torch.randn(nbuf * R, dtype=torch.float64, device="cuda", generator=g)
        sig = clean.repeat(nbuf) + 0.01 * noise
        sig[7 * R: 9 * R] = 0.8 * noise[7 * R: 9 * R]  # two noise-only buffers: status 1/2 + m-grid retry
        recs.append(sig)
    x = torch.stack(recs).contiguous()
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for ladder, split in ((32, 0), (0, 0), (32, 4)):
        _lib.check(lib.dfmi_set_tuning(b"lm_ladder", ladder), "dfmi_set_tuning")
        _lib.check(lib.dfmi_set_tuning(b"lm_ladder_split", split), "dfmi_set_tuning")
        out = []
        for kw in (dict(parallel=False), dict(parallel=True, n_cores=4), dict(parallel=True)):
            cols, ok = nls_records(x, 200000.0, 1000.0, R, nbuf, nd, **kw)
            out += [cols.cpu().numpy(), ok.cpu().numpy()]
        qi = torch.empty((2 * nd, nbuf), dtype=torch.float64, device="cuda")
        dc = torch.empty(nbuf, dtype=torch.float64, device="cuda")
        _lib.check(lib.dfmi_demod(x.data_ptr(), nbuf, R, R, nd, 2 * np.pi * 1000.0 / 200000.0, 0, qi.data_ptr(),
                                  dc.data_ptr(), _lib.DFMI_MEM_DEVICE, st), "dfmi_demod")
        gd = torch.tensor(np.tile([1.0, 6.0, 0.0, 0.0], (nbuf, 1)), dtype=torch.float64, device="cuda")
        p = torch.empty((4, nbuf), dtype=torch.float64, device="cuda")
        ssq = torch.empty(nbuf, dtype=torch.float64, device="cuda")
        stt = torch.empty(nbuf, dtype=torch.int32, device="cuda")
        _lib.check(lib.dfmi_lm(qi.data_ptr(), nbuf, nd, gd.data_ptr(), 1, nbuf, F.lm_config(), p.data_ptr(),
                               ssq.data_ptr(), stt.data_ptr(), _lib.DFMI_MEM_DEVICE, st), "dfmi_lm")
        out += [a.cpu().numpy() for a in (p, ssq, stt)]
        res[(ladder, split)] = out
    one, lad, spl = res[(0, 0)], res[(32, 0)], res[(32, 4)]
    assert any((one[i] != 0).any() for i in (1, 3, 5, 8))  # the m-grid retry path ran (status 1/2)
    for i, (a, b) in enumerate(zip(lad, one)):
        np.testing.assert_array_equal(a, b, err_msg=f"output {i}")
    if nd > 16:  # the wave-split ladder: same statuses, status-0 fits within 1e-7
        for cols_i, ok_i in ((0, 1), (2, 3), (4, 5)):
            np.testing.assert_array_equal(spl[ok_i], one[ok_i])
            good = one[ok_i].reshape(-1) == 0
            d = np.abs(spl[cols_i].reshape(spl[cols_i].shape[0], -1) - one[cols_i].reshape(one[cols_i].shape[0], -1))
            assert d[:4, good].max() <= 1e-7, d[:4, good].max()
        np.testing.assert_array_equal(spl[8], one[8])
        good = one[8] == 0
        assert np.abs(spl[6][:, good] - one[6][:, good]).max() <= 1e-7


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


@pytest.mark.parametrize("method,nb", [(1, 14), (2, 18)])
def test_device_bessel_regs_vs_host_build(method, nb):
    """The register path's Miller pass on the device takes 2/x and 1/S by v_rcp_f64 + two
    Newton steps (lm.h rcp_nr), the host build of the same header (tests/hostcheck) by IEEE
    division: an ulp-level deviation by design. Counted here on 200,000 arguments over the
    fitted range (|x| in [1e-3, 40], both signs): how many J_k differ and by how many ulps,
    so any drift shows up as a number (the fit's parity is gated elsewhere)."""
    import ctypes
    hc_path = os.path.join(os.path.dirname(__file__), "hostcheck", "libhostcheck.so")
    if not os.path.exists(hc_path):
        pytest.skip("hostcheck not built")
    hc = ctypes.CDLL(hc_path)
    hc.hc_bessel_regs.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_void_p]
    rng = np.random.default_rng(11)
    x = rng.uniform(1e-3, 40.0, 200_000) * rng.choice([-1.0, 1.0], 200_000)
    dev = _bessel(x, nb - 1, method).T
    host = np.zeros_like(dev)
    row = np.zeros(nb)
    for i, v in enumerate(x):
        hc.hc_bessel_regs(float(v), nb, row.ctypes.data)
        host[i] = row
    diff = dev != host
    ulps = np.abs(dev - host) / np.spacing(np.abs(host))
    frac = diff.mean()
    print(f"bessel_regs<{nb}> device vs host: {diff.sum()} of {diff.size} values differ ({frac:.3%}), "
          f"max {ulps.max():.1f} ulp")
    assert ulps.max() <= 4.0
    assert frac <= 0.05


@pytest.mark.parametrize("phi,psi,noise_only", [(1.3, 0.4, False), (0.0, 0.0, False), (1.0, 1.0, False),
                                                (0.0, 0.0, True)])
def test_seed_wave_ladder_equals_one_lane_general_fit(phi, psi, noise_only):
    """The record pipeline's seed (buffer 0 of the record, fitted inside the fused seed +
    demodulation launch by a whole wave on the 8-lane lambda ladder, seed.h kSeedFlat) gives
    the bits of the one-lane general-path fit of the same QI (dfmi_demod + dfmi_lm with
    lm_general = 1, lm_ladder = 0): records whose phase the default guess cannot reach
    (psi = 0.4 / 1.0: the descent walks the whole ladder, status 2, m-grid retry) and a
    noise-only seed buffer. The phi = 1.3, psi = 0.4 record's step took 29.6 ms with the
    one-lane seed; it is timed here."""
    import time
    import torch
    import bench
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import w0_of
    from deepfmkit_amd.physics import SnrSpec, synth_snr
    lib = _lib.load()
    R, nseg = 4000, 20000
    dev = torch.device("cuda", 0)
    x = torch.empty(nseg * R, dtype=torch.float64, device=dev)
    synth_snr(SnrSpec(seed=bench.SEED, f_samp=200000.0, f_mod=1000.0, m=6.0, phi=phi, psi=psi, snr_db=40.0), 0,
              nseg * R, out=x)
    if noise_only:
        x[:R] = 0.5 + 0.3 * torch.randn(R, dtype=torch.float64, device=dev, generator=torch.Generator(
            device="cuda").manual_seed(3))
    w0 = w0_of(1000.0, 200000.0)
    g = np.array([1.6, 6.0, 0.0, 0.0])
    st = torch.cuda.current_stream().cuda_stream
    out = torch.empty((6, nseg), dtype=torch.float64, device=dev)
    ok = torch.empty(nseg, dtype=torch.int32, device=dev)

    def step():
        _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nseg * R, nseg, R, 10, w0, 0, _lib.ptr(g), 1, nseg - 1,
                                       F.lm_config(), out.data_ptr(), ok.data_ptr(), _lib.DFMI_MEM_DEVICE, st),
                   "dfmi_nls_record")

    step()
    torch.cuda.synchronize()
    assert lib.dfmi_last_demod_kernel().decode().startswith("demod_seed_bins_kernel")
    t0 = time.perf_counter()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 3 * 1e3
    seed = out[:, 0].cpu().numpy()
    seed_st = int(ok[0].item())
    qi = torch.empty((20, 1), dtype=torch.float64, device=dev)
    dc = torch.empty(1, dtype=torch.float64, device=dev)
    _lib.check(lib.dfmi_demod(x.data_ptr(), 1, R, R, 10, w0, 0, qi.data_ptr(), dc.data_ptr(), _lib.DFMI_MEM_DEVICE,
                              st), "dfmi_demod")
    gd = torch.tensor([1.6, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    p = torch.empty((4, 1), dtype=torch.float64, device=dev)
    ssq = torch.empty(1, dtype=torch.float64, device=dev)
    s1 = torch.empty(1, dtype=torch.int32, device=dev)
    old = {k: np.zeros(1, dtype=np.int64) for k in (b"lm_general", b"lm_ladder")}
    for k in old:
        _lib.check(lib.dfmi_get_tuning(k, _lib.ptr(old[k])), "get")
    try:
        _lib.check(lib.dfmi_set_tuning(b"lm_general", 1), "set")
        _lib.check(lib.dfmi_set_tuning(b"lm_ladder", 0), "set")
        _lib.check(lib.dfmi_lm(qi.data_ptr(), 1, 10, gd.data_ptr(), 0, 1, F.lm_config(), p.data_ptr(), ssq.data_ptr(),
                               s1.data_ptr(), _lib.DFMI_MEM_DEVICE, st), "dfmi_lm")
        torch.cuda.synchronize()
    finally:
        for k, v in old.items():
            _lib.check(lib.dfmi_set_tuning(k, int(v[0])), "set")
    np.testing.assert_array_equal(seed[:4], p[:, 0].cpu().numpy())
    assert seed[5] == ssq[0].item() and seed_st == int(s1[0].item())
    assert seed[4] == dc[0].item()
    print(f"phi={phi} psi={psi} noise_only={noise_only}: seed status {seed_st}, step {ms:.3f} ms "
          f"({nseg} segments)")
    assert ms < 10.0


@pytest.mark.parametrize("method,nmax", [(0, 17), (1, 13), (2, 17)])
def test_device_bessel_large_argument(method, nmax):
    """|x| >= 64 on the device (the Hankel expansion + upward recurrence of dfmi_math.h, in
    the general path's table and both register-path passes) against scipy.special.jv
    (tests/golden/bessel_large.npz; scipy's own error there is ~3.3e-15)."""
    d = np.load(os.path.join(GOLDEN, "bessel_large.npz"))
    x, jv = d["x"], d["jv"][: nmax + 1]
    assert np.abs(_bessel(x, nmax, method) - jv).max() <= 1e-14


@pytest.mark.parametrize("nd", [20, 30, 38, 62])
def test_lm_one_pass_bessel_walk_bit_identical(nd):
    """The general path's one-pass Bessel walk (lm_onepass: the lane's recurrence values kept
    in LDS, lm.h harmonic_walk_q) against the two-pass walk on the same QI: the same bits
    (the stored values are the ones the second pass would form again), for noiseless and
    noisy segments, m small enough to rescale the recurrence (the two-pass fallback) and
    negative m seeds."""
    import torch
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    lib = _lib.load()
    from scipy.special import jv
    rng = np.random.default_rng(nd)
    n = 4096
    j = np.arange(1, nd + 1)
    a = rng.uniform(0.3, 2.0, n)[:, None]
    m = rng.uniform(0.05, 25.0, n)[:, None]
    phi = rng.uniform(-np.pi, np.pi, n)[:, None]
    psi = rng.uniform(-0.5, 0.5, n)[:, None]
    c = a * np.cos(phi + j * np.pi / 2) * jv(j, m)  # the model's QI (fit.py:110-114)
    qi = np.concatenate([c * np.cos(j * psi), -c * np.sin(j * psi)], axis=1)
    qi += rng.normal(size=qi.shape) * 10 ** rng.uniform(-6, -1, (n, 1))
    guess = np.column_stack([np.full(n, 1.6), rng.uniform(-8.0, 30.0, n), np.zeros(n), np.zeros(n)])
    res = {}
    for mode in (2, 0):
        _lib.check(lib.dfmi_set_tuning(b"lm_onepass", mode), "tune")
        try:
            res[mode] = F.fit_batch(nd, qi, guess)
        finally:
            _lib.check(lib.dfmi_set_tuning(b"lm_onepass", 1), "tune")
    for a, b in zip(res[2], res[0]):
        np.testing.assert_array_equal(a, b)
