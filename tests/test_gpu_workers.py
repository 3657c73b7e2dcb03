"""The trial workers (reference workers.py:44-189) against the reference's own
run_efficiency_trial results (tests/golden/workers.json, made by
tests/golden/make_workers_golden.py): one Configure-Simulate-Fit trial per call
(run_efficiency_trial), and the batched form (run_efficiency_trials: every trial a
record of one GPU call, each with its own seed) giving the same bits.

Tolerance: |m - m_ref| <= 1e-9 (status-0 fits)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
G = json.load(open(os.path.join(HERE, "golden", "workers.json")))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def params_of(t):
    import deepfmkit_amd as dfm
    laser = dfm.LaserConfig()
    laser.f_mod = 1000.0
    laser.amp_n = t["amp_n"]
    ifo = dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, t["m_true"])
    assert laser.df == t["df"]
    return dict(laser_config=laser, ifo_config=ifo, n_seconds=t["n_seconds"], ndata=t["ndata"],
                m_true=t["m_true"], trial_num=t["trial_num"])


def test_run_efficiency_trial_matches_reference():
    from deepfmkit_amd import workers
    for t in G["trials"]:
        m = workers.run_efficiency_trial(params_of(t))
        assert abs(m - t["m_fit"]) <= 1e-9, (t, m)


def test_batched_trials_equal_single_trials():
    from deepfmkit_amd import workers
    ps = [params_of(t) for t in G["trials"]]
    batched = workers.run_efficiency_trials(ps)
    single = np.array([workers.run_efficiency_trial(p) for p in ps])
    np.testing.assert_array_equal(batched, single)
    ref = np.array([t["m_fit"] for t in G["trials"]])
    assert np.max(np.abs(batched - ref)) <= 1e-9
