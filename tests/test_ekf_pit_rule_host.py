"""The EKF parallel-in-time stop rule (deepfmkit_amd/csrc/ekf_pit.h pit_decide, the device code
built for the host by tests/hostcheck) on move sequences: synthetic ones whose fixed-point
distance is known, and the measured GPU traces of round 5 (profiles/r05/ekf_pit_rule_probe.jsonl:
every pass's snapshot move, and the true distance of that pass's snapshots from the scalar C
oracle with the rule switched off).

The rule: converged when rho / (1 - rho) * d_k <= tol, rho the larger of the last two trusted
ratios d_k / d_{k-1}; moves at or below tol are rounding (the last trusted ratio stands in);
handed to the sequential kernel (status 2) after stall_max passes in a row whose 4-pass
geometric-mean contraction is >= 1, or >= 0.5 and too slow to meet the bound within the cap,
or at a non-finite move after pass 0."""
import ctypes
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAN = float("nan")


@pytest.fixture(scope="module")
def hc():
    so = os.path.join(ROOT, "tests", "hostcheck", "libhostcheck.so")
    if not os.path.exists(so):
        pytest.skip("tests/hostcheck/libhostcheck.so not built")
    lib = ctypes.CDLL(so)
    P = ctypes.c_void_p
    lib.hc_pit_decide.argtypes = [P, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int, P, P]
    return lib


def decide(hc, moves, tol=1e-13, stall=3, cap=48):
    m = np.ascontiguousarray(moves, dtype=np.float64)
    p, s = ctypes.c_int(), ctypes.c_int()
    hc.hc_pit_decide(m.ctypes.data, m.size, tol, stall, cap, ctypes.byref(p), ctypes.byref(s))
    return p.value, s.value


def geometric(d1, rho, n, floor=0.0, seed=0):
    """Moves of an iteration whose distance from the fixed point is e_k = e_1 rho^(k-1): d_k =
    e_{k-1} - e_k, plus rounding noise of size floor."""
    rng = np.random.default_rng(seed)
    e = d1 / (1 - rho) * rho ** np.arange(n)
    d = np.abs(np.diff(np.concatenate([[e[0] / rho], e])))
    d = np.maximum(d, floor * rng.uniform(0.3, 1.0, n))
    return np.concatenate([[NAN], d[: n - 1]]), e


@pytest.mark.parametrize("rho", [0.01, 0.1, 0.3, 0.45])
def test_contracting_channel_stops_within_the_bound(hc, rho):
    moves, e = geometric(1e-3, rho, 60)
    k, s = decide(hc, moves)
    assert s == 1, (k, s)
    # pass k's snapshots (moves[k-1] is that pass's move): their true distance e[k-2] is
    # within the bound; a pass earlier the bound had not held
    assert e[k - 2] <= 1e-13 * 1.01, (k, e[k - 2])
    assert e[k - 3] > 1e-13 * rho


def test_noise_floor_after_fast_contraction_converges(hc):
    # config 5's measured sequence (profiles/r05/ekf_pit_rule_probe.jsonl): 1.4e-4, 1.3e-7, 6.7e-10,
    # 2.5e-12, 1.4e-13, then the rounding floor ~3e-14
    moves = [NAN, 1.4e-4, 1.3e-7, 6.7e-10, 2.5e-12, 1.4e-13, 7.9e-14, 3.4e-14, 3.2e-14]
    assert decide(hc, moves) == (5, 1)


def test_slow_contraction_beyond_the_cap_is_handed_over(hc):
    moves, _ = geometric(1e-2, 0.8, 60)  # would need ~100 passes
    k, s = decide(hc, moves)
    # judged from pass 16 on (ekf_pit_slow_from: the start-up transient is exempt), 3 in a row
    assert s == 2 and k <= 18, (k, s)


def test_alternating_moves_converge_by_their_envelope(hc):
    """A period-2 component: single-pass ratios alternate above and below 1 while every second
    pass contracts by 0.07 (a well-conditioned stress channel of round 6 ran into the cap this
    way under the ratio bound alone). The envelope bound ends it once 2 D r / (1 - r) <= 1e-13."""
    d = [NAN]
    v = 2.9e-2
    for k in range(40):
        d.append(v if k % 2 == 0 else v * 1.3)  # large, larger, then both shrink
        if k % 2 == 1:
            v *= 0.07
    k, s = decide(hc, d)
    assert s == 1, (k, s)
    # pass k's snapshots (move d[k - 1]) are within the bound of the fixed point: the moves
    # still to come add up to at most 1e-13
    assert sum(d[k:]) <= 1e-13, (k, sum(d[k:]))
    assert sum(d[k - 2:]) > 1e-13  # and the rule did not stop passes early


def test_growing_moves_are_handed_over_early(hc):
    """Not contracting at all (the 4-pass geometric mean >= 1) still counts from the first
    passes: a filter that never locks is handed over within a few passes, grace or not."""
    moves = [NAN] + [0.1 * 1.2 ** k for k in range(30)]
    k, s = decide(hc, moves)
    assert s == 2 and k <= 6, (k, s)


def test_slow_but_feasible_contraction_keeps_passing(hc):
    moves, e = geometric(1e-6, 0.5, 60)  # ~25 passes: within the cap
    k, s = decide(hc, moves)
    assert s == 1 and e[k - 2] <= 1e-13 * 1.01, (k, s)


def test_non_contracting_and_non_finite(hc):
    rng = np.random.default_rng(3)
    moves = np.concatenate([[NAN], rng.uniform(0.4, 2.0, 30)])  # a filter that never locks
    k, s = decide(hc, moves)
    assert s == 2 and k <= 6, (k, s)
    assert decide(hc, [NAN, 1e-3, NAN, 1e-5]) == (3, 2)
    assert decide(hc, [NAN, 0.0]) == (2, 1)  # nothing moved: the fixed point itself


def test_one_small_move_does_not_end_the_passes(hc):
    # a single snapshot crossing its old value: the larger of the last two ratios is used
    moves = [NAN, 1e-3, 5e-4, 2.5e-9, 1.2e-4, 6e-5, 3e-5]
    k, s = decide(hc, moves)
    assert (k, s) != (4, 1)


def test_measured_traces_stop_where_the_true_distance_is_within_the_bound(hc):
    """Each named record of the round-5 probe: the pass the rule picks has snapshots within
    1e-13 (relative) of the fixed point and at most ~2e-13 from the C oracle (rounding of two
    different evaluation orders on top)."""
    path = os.path.join(ROOT, "profiles", "r05", "ekf_pit_rule_probe.jsonl")
    if not os.path.exists(path):
        pytest.skip("no probe record")
    n = 0
    for line in open(path):
        d = json.loads(line)
        if "record" not in d:
            continue
        moves = np.array([NAN if v is None else v for v in d["moves"]])
        errs = np.array(d["err_vs_c_at_pass"])
        k, s = decide(hc, moves)
        if d["record"] == "m20_init6":  # never locks: handed over
            assert s == 2, (d["record"], k, s)
            continue
        assert s == 1, (d["record"], k, s)
        assert errs[k - 1] <= 2e-13, (d["record"], k, errs[k - 1])
        assert d["default_rule"]["passes"] == k  # the GPU made the same decision
        n += 1
    assert n >= 3
