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
