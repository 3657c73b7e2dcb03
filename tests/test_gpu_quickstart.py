"""The reference quickstart's own fit at its own size, on the GPU through the drop-in facade.

notebooks/0.0_quickstart.ipynb cell 0: 10 s at 200 kS/s, 40 dB snr mode, m_target = 10*3.14 via
set_laser_df_for_effect (arms 0.1 / 0.3 m), dff.fit(label, ndata=int(2*m_target)) = ndata 62,
n = 20: 500 buffers of R = 4000. tests/golden/make_quickstart_golden.py ran exactly that through
the reference and stored the outputs (tests/golden/quickstart.npz) and the input's SHA-256
(quickstart.json). Here the package regenerates the record with its own API (the same calls),
checks the SHA, and fits it the four ways the fixture holds, at ndata 62 and 30:

  nb     the notebook's call, DeepFitFramework.fit(label, ndata=nd) with the reference's
         n_cores = os.cpu_count() of the generating container (array_split chains)
  seq    StandardNLSFitter._fit_sequential (fitters.py:370-393)
  c1     _fit_parallel with chunk size 1 (fitters.py:395-428; this package's default split)
  par4   _fit_parallel, n_cores=4

Buffer 0 is fitted from the default m = 6 seed, fails (ssq >= FITOK_THRESHOLD) and takes the
m-grid seed (fit.py:260-361, status 1) before seeding the rest. Gate: status equal everywhere,
status-0 buffers within 1e-9 (record_tol's floor; the 40 dB records' ssq resolution is ~1e-11),
dc relative 1e-13, ssq relative 1e-6; QI and tau against the reference's."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, compare_fit, record_tol, sha

pytestmark = pytest.mark.gpu
COLS = ("amp", "m", "phi", "psi", "dc", "ssq", "fitok")


@pytest.fixture(scope="module")
def quick():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with open(os.path.join(GOLDEN, "quickstart.json")) as f:
        meta = json.load(f)
    return meta, np.load(os.path.join(GOLDEN, "quickstart.npz"))


def quickstart_framework():
    """Cell 0 of the notebook, steps 1-6, with this package's API."""
    import deepfmkit_amd as dfm
    dff = dfm.DeepFitFramework()
    laser = dfm.LaserConfig(label="main_laser")
    laser.f_mod = 1000
    ifo = dfm.InterferometerConfig(label="dynamic_ifo")
    ifo.ref_arml = 0.1
    ifo.meas_arml = 0.3
    m_target = 10 * 3.14
    dfm.set_laser_df_for_effect(laser, ifo, m_target)
    label = "dynamic_channel"
    dff.load_sim(dfm.DFMIObject(label=label, laser_config=laser, ifo_config=ifo, f_samp=200e3))
    dff.simulate(main_label=label, n_seconds=10, mode="snr", snr_db=40)
    return dff, label, m_target


def test_quickstart_input_and_quadratures(quick):
    meta, npz = quick
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import w0_of
    dff, label, m_target = quickstart_framework()
    x = dff.raws[label].samples()
    assert x.size == meta["N"] and sha(x) == meta["sha256"]
    assert int(2 * m_target) == 62
    R, nbuf = meta["R"], meta["nbuf"]
    qi, _ = F.demodulate(x[:nbuf * R].reshape(nbuf, R), 62, w0_of(1000.0, 200000.0))
    assert np.abs(qi - npz["qi62"]).max() <= 1e-12, np.abs(qi - npz["qi62"]).max()


@pytest.mark.parametrize("nd", [62, 30])
@pytest.mark.parametrize("mode", ["nb", "seq", "c1", "par4"])
def test_quickstart_fit(quick, nd, mode):
    meta, npz = quick
    from deepfmkit_amd.fitters import StandardNLSFitter
    dff, label, _ = quickstart_framework()
    raw = dff.raws[label]
    if mode == "nb":
        fobj = dff.fit(label, ndata=nd, n_cores=meta["nb_n_cores"])
        df = dff.fits_df[f"{label}_nls"]
        np.testing.assert_allclose(np.asarray(fobj.tau), npz[f"nd{nd}_nb_tau"], rtol=1e-9, atol=0)
    elif mode == "seq":
        df = StandardNLSFitter({"n": 20}).fit(raw, parallel=False, ndata=nd)
    elif mode == "c1":
        df = StandardNLSFitter({"n": 20}).fit(raw, parallel=True, ndata=nd)
    else:
        df = StandardNLSFitter({"n": 20}).fit(raw, parallel=True, n_cores=4, ndata=nd)
    ours = {k: df[k].to_numpy() for k in COLS}
    ref = {k: npz[f"nd{nd}_{mode}_{k}"] for k in COLS}
    assert ref["fitok"][0] == 1 and ours["fitok"][0] == 1  # buffer 0 through the m-grid seed
    np.testing.assert_array_equal(ours["fitok"], ref["fitok"])
    qi = npz["qi62"] if nd == 62 else np.concatenate([npz["qi62"][:, :30], npz["qi62"][:, 62:92]], axis=1)
    rep = compare_fit(ours, ref, tol=record_tol(nd, qi, ref), min_status_match=1.0)
    print(f"quickstart ndata {nd} {mode}: max |d| amp {rep['amp']:.2e} m {rep['m']:.2e} phi {rep['phi']:.2e} "
          f"psi {rep['psi']:.2e}")


@pytest.mark.parametrize("split", [1, 0])
def test_quickstart_seed_paths(quick, split):
    """Buffer 0's fit beyond 16 harmonics by the whole wave as 8 rungs x 8 harmonic shares
    (seed_wave_split 1, the default: seed.h SFLAT 3, lm.h PartFullEval) and by 8-lane groups
    each running the whole fit (0): both through the m-grid seed (status 1) and every buffer
    within the gates of the reference's chunk-size-1 outputs at ndata 62."""
    meta, npz = quick
    from deepfmkit_amd import _lib
    from deepfmkit_amd.fitters import StandardNLSFitter
    lib = _lib.load()
    dff, label, _ = quickstart_framework()
    _lib.check(lib.dfmi_set_tuning(b"seed_wave_split", split), "tune")
    try:
        df = StandardNLSFitter({"n": 20}).fit(dff.raws[label], parallel=True, ndata=62)
    finally:
        _lib.check(lib.dfmi_set_tuning(b"seed_wave_split", 1), "tune")
    ours = {k: df[k].to_numpy() for k in COLS}
    ref = {k: npz[f"nd62_c1_{k}"] for k in COLS}
    assert ours["fitok"][0] == 1
    np.testing.assert_array_equal(ours["fitok"], ref["fitok"])
    rep = compare_fit(ours, ref, tol=record_tol(62, npz["qi62"], ref), min_status_match=1.0)
    print(f"seed_wave_split {split}: max |d| amp {rep['amp']:.2e} m {rep['m']:.2e} phi {rep['phi']:.2e} "
          f"psi {rep['psi']:.2e}")
