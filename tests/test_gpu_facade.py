"""DeepFitFramework.fit on a record already on the GPU (the device-resident drop-in path,
core.py:424-517 / fitters.py:330-428): the result columns leave the device in one pinned copy
and the DataFrame wraps that memory (fitters.frame_from), so a fit's frame and DeepFitObject
must stay what they were when later fits run (torch's host allocator may hand the same pinned
block to a later call only once nothing references it), and equal the host-record path bit for
bit, with the reference's columns, order and dtypes (tau appended by _finish)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _raw(dfm, data, name):
    raw = dfm.DeepRawObject(data)
    raw.f_samp, raw.f_mod, raw.label = 200000.0, 1000.0, name
    return raw


def test_device_frames_survive_later_fits(torch):
    import deepfmkit_amd as dfm
    from deepfmkit_amd.physics import SnrSpec, synth_snr
    R, nbuf = 4000, 2000
    xs = []
    for k, m in enumerate((6.0, 4.3, 9.0)):
        x = torch.empty(nbuf * R, dtype=torch.float64, device="cuda")
        synth_snr(SnrSpec(seed=77, stream=k, f_samp=200000.0, f_mod=1000.0, m=m, snr_db=40.0), 0, nbuf * R, out=x)
        xs.append(x)
    dff = dfm.DeepFitFramework()
    fits, frames, snaps = [], [], []
    for k, x in enumerate(xs):
        dff.raws[f"r{k}"] = _raw(dfm, x, f"r{k}")
        fo = dff.fit(f"r{k}", n=20)
        df = dff.fits_df[f"r{k}_nls"]
        fits.append(fo)
        frames.append(df)
        snaps.append(df.to_numpy(copy=True))
        assert list(df.columns) == ["amp", "m", "phi", "psi", "dc", "ssq", "fitok", "tau"]
        assert [str(t) for t in df.dtypes] == ["float64"] * 6 + ["int64", "float64"]
        assert fo.time.shape == (nbuf,) and fo.m.shape == (nbuf,)
    for _ in range(3):  # more fits through the same pinned sizes
        dff.fit("r1", n=20, fit_label="again")
    for k, (df, snap, fo) in enumerate(zip(frames, snaps, fits)):
        np.testing.assert_array_equal(df.to_numpy(), snap)
        np.testing.assert_array_equal(fo.m, snap[:, 1])
        assert abs(float(np.mean(fo.m)) - (6.0, 4.3, 9.0)[k]) < 1e-3
    # the same record from host memory: the same bits
    host = dfm.DeepFitFramework()
    host.raws["h"] = _raw(dfm, xs[2].cpu().numpy(), "h")
    host.fit("h", n=20)
    np.testing.assert_array_equal(host.fits_df["h_nls"].to_numpy(), snaps[2])
    t1 = fits[0].time
    t1[0] = -1.0  # every fit object owns its time axis (the cached one is handed out as a copy)
    assert fits[1].time[0] == 0.0


def test_device_record_with_sim_tau_matches_host_and_reference(torch, manifest, records_npz):
    """A simulated record (tau = m / (2 pi df), core.py:506-509, formed inside the fitter's
    prebuilt frame for a device record) fitted from HBM and from host memory: the same frame
    bit for bit, and tau equal to the reference's own facade output (tests/golden)."""
    from conftest import make_record
    e = next(r for r in manifest["records"] if r["name"] == "config1")
    dff = make_record(e)
    raw = dff.raws["config1"]
    dff.fit("config1", n=e["n"], fit_label="host")
    host_df = dff.fits_df["host"]
    raw.data = torch.from_numpy(raw.samples().copy()).to("cuda")
    fo = dff.fit("config1", n=e["n"], fit_label="dev")
    dev_df = dff.fits_df["dev"]
    assert list(dev_df.columns) == list(host_df.columns)
    np.testing.assert_array_equal(dev_df.to_numpy(), host_df.to_numpy())
    np.testing.assert_array_equal(fo.tau, dev_df["tau"].to_numpy())
    np.testing.assert_allclose(fo.tau, records_npz["config1_facade_tau"], rtol=0, atol=1e-18)
