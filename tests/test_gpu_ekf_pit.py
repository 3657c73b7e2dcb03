"""The EKF parallel in time (deepfmkit_amd/csrc/ekf_pit.h) against the sequential lane
kernel and the oracle's scalar C restatement of EKFFitter.fit's loop (fitters.py:274-307,
oracle/csrc/ekf_scalar.c, pinned to the numpy oracle by tests/test_oracle_c.py and to the
reference's own states by tests/test_oracle_golden.py::test_oracle_ekf_full_length).

The parallel form is the sequential filter to rounding (every block runs the true EKF from
an entry state the converged scan supplies), so it is held to the same 1e-12 of the C
oracle as the sequential kernels; a channel that has not converged after the last pass is
re-run by the sequential kernel (the row / lane kernel the sequential path would pick for that
many channels), bit for bit."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QD = np.array([1e-8, 1e-8, 1e-6, 1e-6, 1e-8])


def _raw(dfm, m, seconds, trial, psi=0.0, phi=0.0):
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    laser.psi = psi
    ifo.phi = phi
    dfm.set_laser_df_for_effect(laser, ifo, m)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("p", laser, ifo, f_samp=200000.0))
    dff.simulate("p", n_seconds=seconds, mode="snr", snr_db=40.0, trial_num=trial)
    return np.ascontiguousarray(dff.raws["p"].samples(), dtype=np.float64)


def _c_ekf(x, init4, R, nbuf, qd=QD, r_val=None):
    so = os.path.join(ROOT, "oracle", "libekf_scalar.so")
    if not os.path.exists(so):
        pytest.skip("oracle/libekf_scalar.so not built (make -C oracle)")
    cl = ctypes.CDLL(so)
    P = ctypes.c_void_p
    cl.ekf_scalar.argtypes = [P, ctypes.c_int64, P, P, P, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                              ctypes.c_int64, ctypes.c_int64, P]
    x0 = np.array(list(init4) + [np.mean(x)])
    p0, q = np.ones(5), np.ascontiguousarray(qd, dtype=np.float64)
    st = np.zeros((nbuf, 5))
    cl.ekf_scalar(x.ctypes.data, x.size, x0.ctypes.data, p0.ctypes.data, q.ctypes.data,
                  float(np.var(x) if r_val is None else r_val), 2 * np.pi * 1000.0, 200000.0, R, nbuf, st.ctypes.data)
    return st


class _tune:
    """dfmi_set_tuning for the duration of a block, restoring the defaults."""
    DEFAULTS = {"ekf_row": 1, "ekf_rot": 1, "ekf_pit": 1024, "ekf_pit_min": 4096, "ekf_pit_block": 0,
                "ekf_pit_passes": 0, "ekf_pit_head": 256, "ekf_pit_fused": 1, "ekf_pit_first": 5,
                "ekf_pit_every": 2, "ekf_pit_tol": 13, "ekf_pit_stall": 3, "ekf_pit_trace": 0, "ekf_pit_seq": 1}

    def __init__(self, lib, **kw):
        self.lib, self.kw = lib, kw

    def __enter__(self):
        from deepfmkit_amd import _lib
        for k, v in self.kw.items():
            _lib.check(self.lib.dfmi_set_tuning(k.encode(), v), "tune")
        return self

    def __exit__(self, *exc):
        from deepfmkit_amd import _lib
        for k in self.kw:
            _lib.check(self.lib.dfmi_set_tuning(k.encode(), self.DEFAULTS[k]), "tune")


def _ekf(lib, xs, R, nbuf, init4=(1.6, 6.0, 0.0, 0.0), qd=QD, r_val=None):
    """dfmi_ekf_fit over the records xs (equal lengths, host memory): states (nrec, nbuf, 5),
    the reported kernel and the pass counts."""
    from deepfmkit_amd import _lib
    x = np.ascontiguousarray(np.concatenate(xs), dtype=np.float64)
    n = xs[0].size
    st = np.zeros((len(xs), nbuf, 5))
    i4 = np.array(init4, dtype=np.float64)
    p0, q = np.ones(5), np.ascontiguousarray(qd, dtype=np.float64)
    rv = None if r_val is None else _lib.ptr(np.array([r_val]))
    _lib.check(lib.dfmi_ekf_fit(_lib.ptr(x), len(xs), n, n, _lib.ptr(i4), _lib.ptr(p0), _lib.ptr(q), rv,
                                2 * np.pi * 1000.0, 200000.0, R, nbuf, _lib.ptr(st), _lib.DFMI_MEM_HOST, None),
               "dfmi_ekf_fit")
    kname = lib.dfmi_last_demod_kernel().decode()
    passes = (ctypes.c_int32 * len(xs))()
    _lib.check(lib.dfmi_ekf_pit_passes(ctypes.cast(passes, ctypes.c_void_p), len(xs)), "passes")
    return st, kname, list(passes)


@pytest.fixture(scope="module")
def lib():
    # torch first, as in the other GPU test files (its runtime then owns the device before the
    # library's first call)
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from deepfmkit_amd import _lib
    return _lib.load()


@pytest.fixture(scope="module")
def c5():
    import deepfmkit_amd as dfm
    return _raw(dfm, 6.0, 2.0, 7)


@pytest.mark.parametrize("fused", [1, 0])
def test_pit_config5_default_path_matches_c_oracle(lib, c5, fused):
    """One 400,000-sample channel takes the parallel form by default and converges in a few
    passes — the EKF and the next pass's fold in one kernel (fused, the default) or as separate
    aggregate / blocks kernels; every snapshot within 1e-12 of the C restatement, the sequential
    row kernel within 1e-12 of it too."""
    ref = _c_ekf(c5, (1.6, 6.0, 0.0, 0.0), 4000, 100)
    with _tune(lib, ekf_pit_fused=fused):
        got, kname, passes = _ekf(lib, [c5], 4000, 100)
    assert kname.startswith("ekf_pit"), kname
    assert 1 <= passes[0] <= 8, passes
    err = np.abs(got[0] - ref)
    print("pit passes", passes, "max |d state| vs C oracle", err.max())
    assert err.max() <= 1e-12, (err.max(), np.unravel_index(err.argmax(), err.shape))
    with _tune(lib, ekf_pit=0):
        seq, kseq, ps = _ekf(lib, [c5], 4000, 100)
    assert kseq == "ekf_rot_kernel" and ps == [0]
    assert np.abs(seq[0] - got[0]).max() <= 1e-12


@pytest.mark.parametrize("fused", [1, 0])
@pytest.mark.parametrize("block", [16, 49, 700, 5000])
def test_pit_block_sizes_ragged(lib, block, fused):
    """Block sizes from 16 (2,501 blocks: 40 scan workgroups and a second level) to 5000 (9
    blocks, one workgroup), a 40,003-sample record (no block size divides it), R = 3000
    (snapshots mid-block) and R = 7: all within 1e-12 of the C oracle. (Config 5's 16,000
    blocks in the test above run three levels and the top-down fix-up.)"""
    import deepfmkit_amd as dfm
    x = _raw(dfm, 6.0, 0.2, 3)
    x = np.concatenate([x, x[:3]])
    assert x.size == 40_003
    with _tune(lib, ekf_pit_block=block, ekf_pit_fused=fused):
        for R, nbuf in ((3000, 13), (7, 5714)):
            ref = _c_ekf(x, (1.6, 6.0, 0.0, 0.0), R, nbuf)
            got, kname, passes = _ekf(lib, [x], R, nbuf)
            assert kname.startswith(f"ekf_pit (B={block},"), kname
            assert passes[0] >= 1
            err = np.abs(got[0] - ref).max()
            print("B", block, "R", R, "passes", passes, "err", err)
            assert err <= 1e-12, err


def test_pit_channels_independent(lib):
    """Several channels in one call (different m, phi, psi): at a fixed block size each channel
    equals its own single-channel run bit for bit; at the default block size (which grows with
    the channel count) every channel is within 1e-12 of the C oracle."""
    import deepfmkit_amd as dfm
    xs = [_raw(dfm, 6.0, 0.25, 11), _raw(dfm, 4.3, 0.25, 12, psi=0.3, phi=0.7), _raw(dfm, 9.0, 0.25, 13, phi=1.3)]
    with _tune(lib, ekf_pit_block=25):
        many, kname, passes = _ekf(lib, xs, 4000, 12)
        assert kname.startswith("ekf_pit (B=25,") and all(p >= 1 for p in passes), (kname, passes)
        for c, x in enumerate(xs):
            one, _, _ = _ekf(lib, [x], 4000, 12)
            np.testing.assert_array_equal(many[c], one[0])
    dflt, kname, passes = _ekf(lib, xs, 4000, 12)
    assert kname.startswith("ekf_pit") and all(p >= 1 for p in passes), (kname, passes)
    for c, x in enumerate(xs):
        ref = _c_ekf(x, (1.6, 6.0, 0.0, 0.0), 4000, 12)
        assert np.abs(dflt[c] - ref).max() <= 1e-12


def test_pit_unconverged_falls_back_bit_exact(lib, c5):
    """With one pass allowed the channel has not converged: it is re-run by the sequential
    kernel (ekf_rot_kernel for one channel at R = 4000, on the channel picked into a compact
    buffer), reported as -1 pass, and its states equal that kernel's bit for bit."""
    x = c5[:100_000]
    with _tune(lib, ekf_pit_passes=1):
        got, kname, passes = _ekf(lib, [x], 4000, 25)
    assert kname.startswith("ekf_pit") and kname.endswith("+ ekf_rot_kernel x1") and passes == [-1], (kname, passes)
    with _tune(lib, ekf_pit=0):
        seq, kl, ps = _ekf(lib, [x], 4000, 25)
    assert kl == "ekf_rot_kernel" and ps == [0]
    np.testing.assert_array_equal(got, seq)


def test_pit_fallback_only_for_unconverged_channels(lib):
    """Three channels, one of them made to stall: with the pass cap at 2, every channel is
    handed to the sequential kernel (passes -2); with the defaults, none is. In both, every
    channel equals its own sequential run (the picked channels bit for bit, the converged ones
    to the 1e-12 of the rule)."""
    import deepfmkit_amd as dfm
    xs = [_raw(dfm, 6.0, 0.1, 21), _raw(dfm, 4.3, 0.1, 22, psi=0.3, phi=0.7), _raw(dfm, 9.0, 0.1, 23, phi=1.3)]
    with _tune(lib, ekf_pit=0):
        seq, _, _ = _ekf(lib, xs, 4000, 5)
    with _tune(lib, ekf_pit_passes=2):
        got, kname, passes = _ekf(lib, xs, 4000, 5)
    assert passes == [-2, -2, -2] and kname.endswith("+ ekf_rot_kernel x3"), (kname, passes)
    np.testing.assert_array_equal(got, seq)
    got, kname, passes = _ekf(lib, xs, 4000, 5)
    assert all(p > 0 for p in passes) and "+" not in kname, (kname, passes)
    assert np.abs(got - seq).max() <= 1e-12


def test_pit_trace_and_passes_are_host_side(lib, c5):
    """The pass counts and the per-pass moves are copied to the host by the EKF call itself
    (dfmi_ekf_pit_passes reads no device memory): still readable after the workspaces are
    released, cleared by the next EKF call (zeros after a sequential-path call), and the trace
    ends at the converged pass with a move the rule accepts."""
    import ctypes
    from deepfmkit_amd import _lib
    x = c5[:200_000]
    with _tune(lib, ekf_pit_trace=1):
        _, _, passes = _ekf(lib, [x], 4000, 50)
    tr = np.empty(48)
    _lib.check(lib.dfmi_ekf_pit_trace(tr.ctypes.data, 1, 48), "trace")
    k = passes[0]
    assert k > 1 and np.isnan(tr[0]) and np.isfinite(tr[1:k]).all() and np.isnan(tr[k:]).all(), (k, tr)
    rho = tr[k - 1] / tr[k - 2]
    assert tr[k - 1] == 0 or (rho < 1 and rho / (1 - rho) * tr[k - 1] <= 1e-13) or tr[k - 1] <= 1e-13, tr[:k]
    _lib.check(lib.dfmi_release_workspaces(), "release")
    p2 = (ctypes.c_int32 * 1)()
    _lib.check(lib.dfmi_ekf_pit_passes(ctypes.cast(p2, ctypes.c_void_p), 1), "passes")
    assert list(p2) == [k]
    with _tune(lib, ekf_pit=0):
        _, _, ps = _ekf(lib, [x], 4000, 50)
    assert ps == [0]
    assert lib.dfmi_ekf_pit_trace(tr.ctypes.data, 1, 48) != 0  # no trace kept by that call


def test_pit_tuned_noise_matches_c_oracle(lib):
    """The tuned configuration of the golden set (Q_diag 1e-9/1e-7, R_val 1e-3, m=4.3 record,
    init at the reference defaults): a stiffer filter, still within 1e-12 of the C oracle."""
    import deepfmkit_amd as dfm
    x = _raw(dfm, 4.3, 1.0, 11, psi=0.3, phi=0.7)
    qd = np.array([1e-9, 1e-9, 1e-7, 1e-7, 1e-9])
    ref = _c_ekf(x, (1.6, 6.0, 0.0, 0.0), 4000, 50, qd=qd, r_val=0.001)
    got, kname, passes = _ekf(lib, [x], 4000, 50, qd=qd, r_val=0.001)
    assert kname.startswith("ekf_pit") and passes[0] >= 1, (kname, passes)
    err = np.abs(got[0] - ref).max()
    print("tuned passes", passes, "err", err)
    assert err <= 1e-12, err


def test_pit_nonfinite_channel_is_handed_over(lib):
    """A NaN sample in one of two channels: that filter's states turn NaN from there on, its
    moves are not finite, the rule hands it to the sequential kernel after the first finite-less
    pass (status 2, negative passes) and its states equal the sequential kernel's (NaN where it
    has NaN); the other channel converges as usual and is unaffected (bit-equal to its own run
    at the same block size)."""
    import deepfmkit_amd as dfm
    a = _raw(dfm, 6.0, 0.1, 31)
    b = _raw(dfm, 4.3, 0.1, 32, psi=0.3)
    b_bad = b.copy()
    b_bad[7000] = np.nan
    with _tune(lib, ekf_pit_block=25):
        got, kname, passes = _ekf(lib, [a, b_bad], 4000, 5)
        one, _, _ = _ekf(lib, [a], 4000, 5)
    assert passes[0] > 0 and passes[1] < 0, (kname, passes)
    np.testing.assert_array_equal(got[0], one[0])
    with _tune(lib, ekf_pit=0):
        seq, _, _ = _ekf(lib, [a, b_bad], 4000, 5)
    np.testing.assert_array_equal(got[1], seq[1])
    assert np.isnan(got[1][-1]).any()


def test_pit_record_without_snapshots(lib):
    """n < R (no snapshot to write, nbuf = 0): the call succeeds, every channel reports a
    positive pass count (nothing moves: converged) and nothing is written."""
    import deepfmkit_amd as dfm
    x = _raw(dfm, 6.0, 0.05, 33)[:6000]
    st, kname, passes = _ekf(lib, [x, x], 8000, 0)
    assert st.shape == (2, 0, 5) and kname.startswith("ekf_pit") and all(p > 0 for p in passes), (kname, passes)
