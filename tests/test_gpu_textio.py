"""The raw_data reader's device hand-off (DeepFitFramework.load_raw(device=...),
core.py:259-286 + textio.read_raw): the channels land in HBM bit-identical to the
host read, and the readout of the device-resident record equals the host-loaded
one's bit for bit (the engine runs the same kernels on the same bytes)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_load_raw_to_device_then_fit(tmp_path):
    import torch

    import deepfmkit_amd as dfm
    from deepfmkit_amd import textio
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("s", laser, ifo, f_samp=200000.0))
    dff.simulate("s", n_seconds=0.2, mode="snr", snr_db=40.0, trial_num=3)
    x = np.asarray(dff.raws["s"].samples())
    path = str(tmp_path / "raw.txt")
    textio.write_raw(path, [x, 0.5 * x], 0, 200000.0, 1000.0)

    host = dfm.DeepFitFramework()
    host.load_raw(path, labels=["a", "b"])
    dev = dfm.DeepFitFramework()
    dev.load_raw(path, labels=["a", "b"], device="cuda:0")
    for lab in ("a", "b"):
        hx = np.asarray(host.raws[lab].samples())
        dx = dev.raws[lab].samples()
        assert isinstance(dx, torch.Tensor) and dx.is_cuda
        np.testing.assert_array_equal(dx.cpu().numpy(), hx)
        fh = host.fit(lab, n=20, parallel=True)
        fd = dev.fit(lab, n=20, parallel=True)
        for k in ("amp", "m", "phi", "psi", "dc", "ssq"):
            np.testing.assert_array_equal(np.asarray(getattr(fd, k)), np.asarray(getattr(fh, k)))
