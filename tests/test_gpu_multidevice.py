"""One record's parallel fit spread over several GPUs of one process
(fitters.nls_record_devices, StandardNLSFitter.fit(..., devices=[...]); SURVEY.md §8(e):
contiguous shards, every shard refits the seed buffer, no exchange). On a one-GPU box the
shards share cuda:0 (the same code path: per-shard copies, per-shard records, enqueue all
then gather): the union must equal the single-call fit bit for bit, for host and device
input, shard counts that do and do not divide the buffers, and 1- and 2-buffer records."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

COLS = ("amp", "m", "phi", "psi", "dc", "ssq", "fitok")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _raw(nbuf, on_device):
    import torch
    import deepfmkit_amd as dfm
    from deepfmkit_amd.physics import SnrSpec, synth_snr
    x = synth_snr(SnrSpec(seed=77, m=6.0, snr_db=40.0), 0, nbuf * 4000,
                  out=torch.empty(nbuf * 4000, dtype=torch.float64, device="cuda"))
    raw = dfm.DeepRawObject(x if on_device else x.cpu().numpy())
    raw.f_samp, raw.f_mod = 200000.0, 1000.0
    return raw


@pytest.mark.parametrize("on_device", [False, True])
@pytest.mark.parametrize("nbuf,ndev", [(1001, 3), (1001, 4), (2, 3), (1, 2), (64, 8)])
def test_sharded_fit_equals_single_call(on_device, nbuf, ndev):
    import deepfmkit_amd as dfm
    raw = _raw(nbuf, on_device)
    one = dfm.fitters.StandardNLSFitter({"n": 20}).fit(raw, parallel=True)
    many = dfm.fitters.StandardNLSFitter({"n": 20}).fit(raw, parallel=True, devices=[0] * ndev)
    assert len(many) == nbuf
    for k in COLS:
        np.testing.assert_array_equal(many[k].to_numpy(), one[k].to_numpy(), err_msg=k)


def test_facade_devices_kwarg():
    """DeepFitFramework.fit forwards devices= to the fitter (core.py:424-517 kwargs)."""
    import deepfmkit_amd as dfm
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("r", laser, ifo, f_samp=200000.0))
    dff.simulate("r", n_seconds=1.0, mode="snr", snr_db=40.0, trial_num=3)
    a = dff.fit("r", n=20, fit_label="a")
    b = dff.fit("r", n=20, fit_label="b", devices=[0, 0])
    for k in ("amp", "m", "phi", "psi", "dc", "ssq"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k))


def test_devices_rejected_where_they_would_be_ignored():
    """devices= spreads the chunk-size-1 parallel fit only; with parallel=False or n_cores
    (warm-start chains on one GPU) it is an error, not a silently ignored argument."""
    import deepfmkit_amd as dfm
    raw = _raw(8, False)
    f = dfm.fitters.StandardNLSFitter({"n": 20})
    with pytest.raises(ValueError, match="devices="):
        f.fit(raw, parallel=False, devices=[0])
    with pytest.raises(ValueError, match="devices="):
        f.fit(raw, parallel=True, n_cores=2, devices=[0])


def test_sharded_fit_on_distinct_devices():
    """Two distinct GPUs (skipped on a one-GPU box): the record lives on cuda:1, shards on
    [0, 1]; the union equals the one-GPU fit bit for bit."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    import deepfmkit_amd as dfm
    from deepfmkit_amd.physics import SnrSpec, synth_snr
    nbuf = 2001
    x1 = synth_snr(SnrSpec(seed=78, m=6.0, snr_db=40.0), 0, nbuf * 4000,
                   out=torch.empty(nbuf * 4000, dtype=torch.float64, device="cuda:1"))
    raw = dfm.DeepRawObject(x1)
    raw.f_samp, raw.f_mod = 200000.0, 1000.0
    with torch.cuda.device(1):  # the single-call fit where the record lives
        one = dfm.fitters.StandardNLSFitter({"n": 20}).fit(raw, parallel=True)
    many = dfm.fitters.StandardNLSFitter({"n": 20}).fit(raw, parallel=True, devices=[0, 1])
    for k in COLS:
        np.testing.assert_array_equal(many[k].to_numpy(), one[k].to_numpy(), err_msg=k)
