"""Host-side logic of the Experiment runner (deepfmkit_amd/experiments.py): job list and
stochastic draw order, parameter validation, get_params_for_point, aggregation —
reference experiments.py:127-458. No GPU (the fits run in tests/test_gpu_experiments.py)."""
import itertools

import numpy as np
import pytest

from deepfmkit_amd import factories, physics
from deepfmkit_amd.experiments import Experiment


class KeyFactory(factories.ExperimentFactory):
    def _get_expected_params_keys(self):
        return {"a", "b", "s", "t"}

    def __call__(self, params):
        return {"laser_config": physics.LaserConfig(), "main_ifo_config": physics.InterferometerConfig()}


def _exp():
    e = Experiment("x")
    e.set_config_factory(KeyFactory())
    e.add_axis("a", [1.0, 2.0, 3.0])
    e.add_axis("b", [10.0, 20.0])
    e.set_static({"t": 5})
    e.add_stochastic_variable("s", lambda a: a + np.random.uniform(), depends_on="a")
    e.n_trials = 4
    return e


def test_job_list_order_and_draws():
    """experiments.py:326-375: itertools.product over the axes, n_trials per point, the
    stochastic variables drawn per trial in that order from numpy's global state."""
    e = _exp()
    np.random.seed(3)
    jobs = e._job_list()
    np.random.seed(3)
    want = []
    for (i, j) in itertools.product(range(3), range(2)):
        for k in range(4):
            want.append(((i, j), k, [1.0, 2.0, 3.0][i] + np.random.uniform()))
    assert [num for _, num in jobs] == list(range(24))
    for (p, _), (pt, tr, s) in zip(jobs, want):
        assert p["_exp_point_idx"] == pt and p["_exp_trial_idx"] == tr and p["s"] == s and p["t"] == 5
        assert set(p) == {"a", "b", "s", "t", "_exp_point_idx", "_exp_trial_idx"}


def test_validation_and_point_params():
    e = _exp()
    with pytest.raises(ValueError, match="not recognized"):
        e.add_axis("nope", [1])
    with pytest.raises(TypeError):
        e.set_config_factory(object())
    st = np.random.get_state()
    p1 = e.get_params_for_point((1, 0))
    p2 = e.get_params_for_point((1, 0))
    assert p1 == p2 and p1["a"] == 2.0 and p1["b"] == 10.0
    np.random.seed(0)
    assert p1["s"] == 2.0 + np.random.uniform()
    np.random.set_state(st)
    with pytest.raises(ValueError, match="Dimension"):
        e.get_params_for_point(1)
    with pytest.raises(ValueError, match="configuration factory"):
        Experiment().run()


def test_aggregation_statistics():
    """experiments.py:386-447: all_trials grid, nan-aware mean/std/min/max and the
    worst case (largest deviation from the mean)."""
    e = _exp()
    e.analyses = [{"name": "A", "fitter_method": "nls", "result_cols": None, "fitter_kwargs": {}}]
    np.random.seed(0)
    jobs = e._job_list()
    rng = np.random.default_rng(1)
    vals = rng.normal(size=len(jobs))
    flat = [{"point_params": p, "results": {"A": ({"m": float(v), "x": 1.0} if n != 5 else {})}}
            for (p, n), v in zip(jobs, vals)]
    res = e._aggregate(flat)
    grid = vals.reshape(3, 2, 4).copy()
    grid.reshape(-1)[5] = np.nan  # job 5 (point (0, 1), trial 1) returned no results
    a = res["A"]["m"]["all_trials"]
    np.testing.assert_array_equal(np.isnan(a), np.isnan(grid))
    np.testing.assert_allclose(res["A"]["m"]["mean"], np.nanmean(grid, -1))
    np.testing.assert_allclose(res["A"]["m"]["std"], np.nanstd(grid, -1))
    dev = np.abs(grid - np.nanmean(grid, -1)[..., None])
    worst = np.take_along_axis(grid, np.nanargmax(dev, -1)[..., None], -1)[..., 0]
    np.testing.assert_array_equal(res["A"]["m"]["worst"], worst)
    assert sorted(res["A"]) == ["m", "x"] and res["axes"] is e.axes
