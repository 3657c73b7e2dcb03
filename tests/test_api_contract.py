"""CPU checks of the drop-in API's error contract and of the sharded-record plumbing
(no GPU needed: these paths raise or plan before any engine call).

- ValueError when the record length is not a multiple of R: the reference reshapes
  the whole column with reshape(-1, R) (fitters.py:375, 412); here on the PRODUCT
  path (StandardNLSFitter.fit, DeepFitFramework.fit_many, workers.run_efficiency_trials),
  not only on the oracle (tests/test_oracle_golden.py).
- BaseFitter without 'n' raises ValueError (fitters.py:171-184).
- The counter-based generator's Philox4x32-10 restatement (oracle/philox.py) against
  the Random123 known-answer vectors, and bench.py's config-4 shard plan.
"""
import numpy as np
import pytest

import deepfmkit_amd as dfm
from deepfmkit_amd.data import DeepRawObject


def _raw(n, label="ch"):
    raw = DeepRawObject(data=np.ones(n))
    raw.label, raw.f_samp, raw.f_mod, raw.t0 = label, 200000.0, 1000.0, 0
    return raw


def test_fitter_requires_n():
    with pytest.raises(ValueError, match="'n'"):
        dfm.StandardNLSFitter({})


@pytest.mark.parametrize("parallel", [True, False])
def test_standard_nls_ragged_record_raises(parallel):
    # R = 4000 at n = 20; 2.5 buffers -> reshape(-1, 4000) fails in the reference
    with pytest.raises(ValueError, match="cannot reshape array of size 10000 into shape"):
        dfm.StandardNLSFitter({"n": 20}).fit(_raw(10000), parallel=parallel)


def test_fit_many_ragged_record_raises():
    dff = dfm.DeepFitFramework()
    dff.raws["a"], dff.raws["b"] = _raw(10000, "a"), _raw(10000, "b")
    with pytest.raises(ValueError, match="cannot reshape"):
        dff.fit_many(["a", "b"], n=20)


def test_fit_short_record_returns_none():
    # nbuf == 0: the reference logs an error and returns an empty DataFrame -> fit() None
    dff = dfm.DeepFitFramework()
    dff.raws["a"] = _raw(100, "a")
    assert dff.fit("a", n=20) is None


def test_efficiency_trials_ragged_raises():
    from deepfmkit_amd import workers
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    # n = int(1000 * 0.0105) = 10 -> R = 2000, N = 2100: run_efficiency_trial raises
    p = {"laser_config": laser, "ifo_config": ifo, "n_seconds": 0.0105, "ndata": 10, "m_true": 6.0,
         "trial_num": 0}
    with pytest.raises(ValueError, match="cannot reshape array of size 2100 into shape"):
        workers.run_efficiency_trials([p])


def test_philox_known_answers():
    """Random123 kat_vectors for philox4x32_10."""
    from oracle.philox import philox4x32_10

    def h(c):
        return [int(v) for v in c]

    assert h(philox4x32_10(0, 0, 0, 0, 0, 0)) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    f = 0xFFFFFFFF
    assert h(philox4x32_10(f, f, f, f, f, f)) == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert h(philox4x32_10(0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0)) == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_philox_normals_are_standard_and_split_invariant():
    from oracle.philox import normals
    z = normals(1234, 0, 0, 200_000)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
    # a window regenerated alone equals the same samples of a longer draw (any split, odd starts)
    np.testing.assert_array_equal(normals(1234, 0, 777, 1001), z[777:1778])
    assert not np.array_equal(normals(1234, 1, 0, 100), z[:100])  # streams differ


def test_snr_spec_noise_std_matches_reference_formula():
    """physics.py:520-530 over a whole record of complete modulation cycles equals the
    one-cycle value SnrSpec uses."""
    from deepfmkit_amd.physics import SnrSpec
    s = SnrSpec(m=6.0, snr_db=40.0)
    assert s.period == 200
    t = np.arange(20 * 4000) / 200000.0
    clean = 1.0 * (1 + np.cos(0.0 + 6.0 * np.cos(2 * np.pi * 1000.0 * t)))
    ac = clean - clean.mean()
    ref = np.sqrt(np.mean(ac ** 2) / 10 ** 4.0)
    assert abs(s.noise_std() - ref) <= 1e-15 * ref


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_config4_shards_cover_the_record_once(world):
    import bench
    nseg = bench.CONFIG4_SEGMENTS // world
    seen = 0
    for r in range(world):
        s0, nbuf, pre = bench.shard_plan(r, world, nseg)
        assert s0 == seen and nbuf == nseg + (1 if pre else 0) and pre == (r > 0)
        seen += nseg
    assert seen == bench.CONFIG4_SEGMENTS


def test_cpu_share_reports_host():
    import bench
    share, host = bench.cpu_share()
    assert 1 <= share <= (host["os_cpu_count"] or share)
    assert set(host) >= {"os_cpu_count", "affinity", "cgroup_quota", "model"}
