"""The many-harmonic demodulation (demod.h demod_wide_kernel: ndata beyond the bin kernel's
LDS basis, component-major QI) against the fold / bin kernels and a torch fp64 restatement
of calculate_quadratures (fit.py:18-66: mean(x cos((n+1) w0 t)), mean(x sin(...)), and
fitters.py:57's dc = mean(x)), on ragged shapes: segment counts that leave partial groups,
R with a partial last chunk, basis periods 128..256 (KSEG 8 and 4), 1..3 output slices, and
the flat multi-segment fold of contiguous short segments."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from deepfmkit_amd import _lib
    return torch, _lib, _lib.load()


def _demod(env, x, nseg, R, nd, w0, **tune):
    torch, _lib, lib = env
    for k, v in tune.items():
        _lib.check(lib.dfmi_set_tuning(k.encode(), v), "tune")
    try:
        qi = torch.full((2 * nd, nseg), float("nan"), dtype=torch.float64, device="cuda")
        dc = torch.full((nseg,), float("nan"), dtype=torch.float64, device="cuda")
        _lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0, 0, qi.data_ptr(), dc.data_ptr(),
                                  _lib.DFMI_MEM_DEVICE, torch.cuda.current_stream().cuda_stream), "dfmi_demod")
        torch.cuda.synchronize()
        return qi.cpu().numpy(), dc.cpu().numpy(), lib.dfmi_last_demod_kernel().decode()
    finally:
        for k in tune:
            _lib.check(lib.dfmi_set_tuning(k.encode(), {"demod_wide": 1, "demod_wide_k": 0, "demod_wide_from": 13,
                                                         "demod_wide_dbg": 0, "demod_wide_half": 1}[k]), "tune")


def _torch_ref(torch, x, nseg, R, nd, w0, take):
    """fit.py:18-66 in torch fp64 on the device: the reference's angle fl(fl(h w0) t)."""
    xs = x.view(nseg, R)[take]
    t = torch.arange(R, dtype=torch.float64, device="cuda")
    q, i = [], []
    for h in range(1, nd + 1):
        ang = (h * w0) * t
        q.append((xs * torch.cos(ang)).mean(dim=1))
        i.append((xs * torch.sin(ang)).mean(dim=1))
    return torch.stack(q + i).cpu().numpy(), xs.mean(dim=1).cpu().numpy()


@pytest.mark.parametrize("nd,f_samp,nseg,R", [
    (20, 200000.0, 3001, 4000),   # L 200, one output slice, KSEG 8, partial groups
    (30, 200000.0, 517, 4000),
    (62, 200000.0, 1029, 4000),   # two slices (125 outputs)
    (100, 200000.0, 131, 4000),   # four slices
    (40, 250000.0, 700, 5000),    # L 250: KSEG 4
    (40, 128000.0, 33, 3968),     # L 128, R = 31 chunks exactly
    (20, 200000.0, 5, 4000),      # fewer segments than one group
    (20, 200000.0, 1, 334),       # one segment, shorter than one basis period
])
def test_wide_matches_fold_and_torch_reference(env, nd, f_samp, nseg, R):
    torch = env[0]
    w0 = 2 * np.pi * 1000.0 / f_samp
    g = torch.Generator(device="cuda")
    g.manual_seed(nd * 7919 + nseg)
    x = torch.randn(nseg * R, dtype=torch.float64, device="cuda", generator=g) + 0.25
    qw, dw, kw = _demod(env, x, nseg, R, nd, w0)
    assert kw.startswith("demod_wide_kernel"), kw
    qf, df, kf = _demod(env, x, nseg, R, nd, w0, demod_wide=0)
    assert not kf.startswith("demod_wide"), kf
    scale = np.abs(qf).max()
    assert np.isfinite(qw).all() and np.isfinite(dw).all()
    # half-period pairing: the basis at L - p taken equal to that at p (~h L w0 eps apart)
    assert np.abs(qw - qf).max() <= 1e-13 * max(scale, 1.0), np.abs(qw - qf).max()
    assert np.abs(dw - df).max() <= 1e-14 * max(np.abs(df).max(), 1.0)
    take = torch.arange(0, nseg, max(1, nseg // 24), device="cuda")
    rq, rd = _torch_ref(torch, x, nseg, R, nd, w0, take)
    idx = take.cpu().numpy()
    assert np.abs(qw[:, idx] - rq).max() <= 1e-12, np.abs(qw[:, idx] - rq).max()
    assert np.abs(dw[idx] - rd).max() <= 1e-13
    # other group sizes give the same bits: a segment's result does not depend on the group
    # it is contracted in
    for k in (2, 8):
        qp, dp, _ = _demod(env, x, nseg, R, nd, w0, demod_wide_k=k)
        np.testing.assert_array_equal(qp, qw)
        np.testing.assert_array_equal(dp, dw)


@pytest.mark.parametrize("nd,R,nseg", [(10, 200, 4099), (20, 300, 777), (20, 100, 1001), (30, 1000, 513),
                                        (15, 4000, 67)])
def test_flat_fold_equals_per_segment_fold(env, nd, R, nseg):
    """Contiguous segments are folded as one flat stream per wave (demod_wide_fold_flat):
    the same bits as the segment-by-segment fold (demod_wide_dbg bit 2), for segments
    shorter than a chunk (R = 100), not a whole number of periods (R = 300, L = 200), and
    long; and the reference's quadratures."""
    torch = env[0]
    w0 = 2 * np.pi * 1000.0 / 200000.0
    g = torch.Generator(device="cuda")
    g.manual_seed(R + nd)
    x = torch.randn(nseg * R, dtype=torch.float64, device="cuda", generator=g) + 0.5
    qf, df, kf = _demod(env, x, nseg, R, nd, w0)
    assert kf.startswith("demod_wide_kernel"), kf  # R < 2000 or ndata >= 13
    qs, ds, _ = _demod(env, x, nseg, R, nd, w0, demod_wide_dbg=4)
    np.testing.assert_array_equal(qf, qs)
    np.testing.assert_array_equal(df, ds)
    # the half-wave contraction (2 ndata + 1 <= 32: each half-wave its own segments) is the
    # same fma chain per output: the same bits with it off
    qh, dh, kh = _demod(env, x, nseg, R, nd, w0, demod_wide_half=0)
    assert kf.endswith(",1>") == (2 * nd + 1 <= 32) and kh.endswith(",0>"), (kf, kh)
    np.testing.assert_array_equal(qf, qh)
    np.testing.assert_array_equal(df, dh)
    take = torch.arange(0, nseg, max(1, nseg // 16), device="cuda")
    rq, rd = _torch_ref(torch, x, nseg, R, nd, w0, take)
    idx = take.cpu().numpy()
    assert np.abs(qf[:, idx] - rq).max() <= 1e-12
    assert np.abs(df[idx] - rd).max() <= 1e-13


@pytest.mark.parametrize("nd", [10, 12, 16])
def test_wide_forced_at_bin_kernel_ndata(env, nd):
    """demod_wide = 2 runs the many-harmonic kernel where the bin kernel also applies (A/B; by
    default it takes over from 13 harmonics): the same QI within a few ulps."""
    torch = env[0]
    w0 = 2 * np.pi * 1000.0 / 200000.0
    g = torch.Generator(device="cuda")
    g.manual_seed(nd)
    nseg, R = 2049, 4000
    x = torch.randn(nseg * R, dtype=torch.float64, device="cuda", generator=g) - 0.5
    qb, db, kb = _demod(env, x, nseg, R, nd, w0, demod_wide=0)
    assert kb.startswith("demod_bins_kernel"), kb
    qw, dw, kw = _demod(env, x, nseg, R, nd, w0, demod_wide=2)
    assert kw.startswith("demod_wide_kernel"), kw
    assert np.abs(qw - qb).max() <= 1e-13 * max(np.abs(qb).max(), 1.0)
    assert np.abs(dw - db).max() <= 1e-14


@pytest.mark.parametrize("nd", [12, 13, 16])
def test_record_pipeline_switches_layout_at_wide_from(env, nd):
    """ndata >= demod_wide_from (13): the record pipeline leaves the row layout and the fused
    seed launch for component-major QI through demod_wide_kernel (seed on the side stream);
    below it the fused bin kernel stays. Noiseless m = 6 segments are recovered either way,
    and the two layouts agree to the parity tolerance."""
    torch, _lib, lib = env
    from deepfmkit_amd.fitters import nls_records
    nseg, R = 3000, 4000
    t = torch.arange(R, dtype=torch.float64, device="cuda") / 200000.0
    seg_phi = torch.linspace(-0.4, 0.4, nseg, dtype=torch.float64, device="cuda")
    x = (1.0 + torch.cos(seg_phi[:, None] + 6.0 * torch.cos(2 * np.pi * 1000.0 * t[None, :] + 0.1))).reshape(1, -1)
    cols, ok = nls_records(x, 200000.0, 1000.0, R, nseg, nd)
    k = lib.dfmi_last_demod_kernel().decode()
    assert k.startswith("demod_wide_kernel" if nd >= 13 else "demod_seed_bins_kernel"), (nd, k)
    _lib.check(lib.dfmi_set_tuning(b"demod_wide_from", 1000), "tune")
    try:
        cols2, ok2 = nls_records(x, 200000.0, 1000.0, R, nseg, nd)
        assert lib.dfmi_last_demod_kernel().decode().startswith("demod_seed_bins_kernel")
    finally:
        _lib.check(lib.dfmi_set_tuning(b"demod_wide_from", 13), "tune")
    cols, ok, cols2, ok2 = (a.cpu().numpy() for a in (cols, ok, cols2, ok2))
    assert (ok == 0).all() and (ok2 == 0).all()
    assert np.abs(cols[1] - 6.0).max() < 1e-9
    assert np.abs(cols[:4] - cols2[:4]).max() < 1e-9


def test_record_pipeline_at_many_harmonics(env):
    """dfmi_nls_record at ndata 30 (the quickstart's m = 31.4 setting) on a
    noiseless m = 12, psi = 0.2 record seeded near psi (from psi = 0 the LM settles in a local
    minimum at m = 11.2 whichever demodulation runs): every segment recovers the parameters,
    through the many-harmonic demodulation."""
    torch, _lib, lib = env
    from deepfmkit_amd.fitters import nls_records
    nseg, R = 4000, 4000
    t = torch.arange(R, dtype=torch.float64, device="cuda") / 200000.0
    seg_phi = torch.linspace(-0.4, 0.4, nseg, dtype=torch.float64, device="cuda")
    x = (1.0 + torch.cos(seg_phi[:, None] + 12.0 * torch.cos(2 * np.pi * 1000.0 * t[None, :] + 0.2))).reshape(1, -1)
    cols, ok = nls_records(x, 200000.0, 1000.0, R, nseg, 30, init_guess=(1.6, 12.0, 0.0, 0.2))
    assert lib.dfmi_last_demod_kernel().decode().startswith("demod_wide_kernel")
    cols, ok = cols.cpu().numpy(), ok.cpu().numpy()
    assert (ok == 0).all()
    assert np.abs(cols[0] - 1.0).max() < 1e-9
    assert np.abs(cols[1] - 12.0).max() < 1e-9
    assert np.abs(cols[3] - 0.2).max() < 1e-9


@pytest.mark.parametrize("nd,R", [(20, 4000), (10, 200), (15, 400)])
def test_nonfinite_samples_through_the_wide_path(env, nd, R):
    """Erasures in the many-harmonic / short-segment record path: a NaN or inf sample poisons
    exactly its own segment (every QI of it, through the bins' half-period pairing and the
    flat multi-segment fold) as it does on the bin / fold kernels: status and every finite
    result agree with demod_wide = 0 (parity 1e-9), the neighbours untouched."""
    torch, _lib, lib = env
    from deepfmkit_amd.fitters import nls_records
    nseg = 2000
    t = torch.arange(R, dtype=torch.float64, device="cuda") / 200000.0
    seg_phi = torch.linspace(-0.3, 0.3, nseg, dtype=torch.float64, device="cuda")
    x = 1.0 + torch.cos(seg_phi[:, None] + 6.0 * torch.cos(2 * np.pi * 1000.0 * t[None, :] + 0.1))
    g = torch.Generator(device="cuda")
    g.manual_seed(R + nd)
    x = (x + 1e-3 * torch.randn(x.shape, dtype=torch.float64, device="cuda", generator=g)).reshape(1, -1)
    bad = {17: float("nan"), 555: float("inf"), 1999: float("-inf")}
    for s_, v in bad.items():
        x[0, s_ * R + R // 3] = v
    cols, ok = nls_records(x, 200000.0, 1000.0, R, nseg, nd)
    k = lib.dfmi_last_demod_kernel().decode()
    assert k.startswith("demod_wide_kernel"), k
    _lib.check(lib.dfmi_set_tuning(b"demod_wide", 0), "tune")
    try:
        cols0, ok0 = nls_records(x, 200000.0, 1000.0, R, nseg, nd)
        assert not lib.dfmi_last_demod_kernel().decode().startswith("demod_wide")
    finally:
        _lib.check(lib.dfmi_set_tuning(b"demod_wide", 1), "tune")
    cols, ok, cols0, ok0 = (a.cpu().numpy() for a in (cols, ok, cols0, ok0))
    np.testing.assert_array_equal(ok, ok0)
    for s_ in bad:
        assert not np.isfinite(cols[4, s_])  # dc of the poisoned segment
    good = np.array([i for i in range(nseg) if i not in bad])
    assert (ok[good] == 0).all()
    assert np.abs(cols[:4, good] - cols0[:4, good]).max() < 1e-9


@pytest.mark.parametrize("parallel", [False, True])
def test_crlb_notebook_call_shape_vs_oracle(env, parallel):
    """notebooks/1.1_CRLB-test's fitter call, StandardNLSFitter({'n': 1, 'ndata': 15}).fit(raw,
    parallel=False) (1-cycle segments, 15 harmonics: demod_wide_kernel and the 16-harmonic LM),
    and its parallel form, on a 40 dB snr-mode record of 0.1 s (100 segments) against the numpy
    oracle (fitters.py:370-393 sequential / 395-428 parallel with chunk size 1): status equal,
    parameters within 1e-9 (a warm-start chain carries each fit into the next one's seed)."""
    import deepfmkit_amd as dfm
    from deepfmkit_amd.fitters import StandardNLSFitter
    from oracle import nls_oracle as O
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("crlb", laser, ifo, f_samp=200000.0))
    dff.simulate("crlb", n_seconds=0.1, mode="snr", snr_db=40.0, trial_num=3)
    raw = dff.raws["crlb"]
    x = np.ascontiguousarray(raw.samples(), dtype=np.float64)
    df = StandardNLSFitter({"n": 1, "ndata": 15}).fit(raw, parallel=parallel)
    if parallel:  # _fit_parallel with chunk size 1, in this process (no Pool from a GPU process)
        R = x.size // 100
        first = O.fit_record_sequential(x[:R], raw.f_samp, raw.f_mod, 1, ndata=15)
        seed = [float(v) for v in first[0, :4]]
        bufs = x.reshape(-1, R)
        ref = np.concatenate([first] + [O.fit_chunk((bufs[b:b + 1], seed, 15, raw.f_mod, raw.f_samp, dict(O.C0)))
                                        for b in range(1, 100)], axis=0)
    else:
        ref = O.fit_record_sequential(x, raw.f_samp, raw.f_mod, 1, ndata=15)
    assert len(df) == ref.shape[0] == 100
    np.testing.assert_array_equal(df["fitok"].to_numpy(), ref[:, 6].astype(int))
    got = np.stack([df[c].to_numpy() for c in ("amp", "m", "phi", "psi")], axis=1)
    d = np.abs(got - ref[:, :4])
    d[:, 2] = np.abs((got[:, 2] - ref[:, 2] + np.pi) % (2 * np.pi) - np.pi)
    assert d.max() <= 1e-9, (int(np.argmax(d.max(axis=1))), d.max(axis=0))
