"""Parity of LM fits against the numpy oracle (oracle/nls_oracle.py fit_segment = the reference's
fit.fit, fit.py:322-361, bit-exact on its golden vectors), for tests/test_gpu_lm_stress.py.

For an ill-conditioned fit that ends at the noise floor, the reference's own answer moves when
its input QI moves by one ulp: the last accept decisions (ssq_try < ssq0, fit.py:240) compare
numbers that differ in their last bits. oracle_spread measures that: the oracle rerun on QI
scaled by (1 +- 2^-52) (fixed random signs, `trials` draws), the largest move of its answer.
A fit beyond the resolution bound (conftest.resolution_tol) of the oracle but within 1.5x that
spread lands where the reference itself lands for an input one ulp away: its distance is the
reference's indeterminacy, not an error of the fit."""
import numpy as np


def _dist(a, b):
    d = np.abs(np.asarray(a, dtype=np.float64) - np.asarray(b, dtype=np.float64))
    d[..., 2] = np.abs((a[..., 2] - b[..., 2] + np.pi) % (2 * np.pi) - np.pi)
    return d


def oracle_fit(args):
    """(ndata, qi, guess) -> (status, p (4,), resolution tolerance (4,))."""
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(os.path.dirname(here)), os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    from conftest import resolution_tol
    from oracle import nls_oracle as O
    nd, qi, g = args
    st, p, _ = O.fit_segment(nd, np.asarray(qi, dtype=np.float64), np.array(g, dtype=np.float64))
    return int(st), np.asarray(p, dtype=np.float64), resolution_tol(nd, qi, p)


def oracle_spread(args):
    """(ndata, qi, guess, p_oracle, trials) -> the oracle's largest move (4,) under one-ulp QI
    perturbations."""
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (os.path.dirname(os.path.dirname(here)), os.path.dirname(here)):
        if p not in sys.path:
            sys.path.insert(0, p)
    from oracle import nls_oracle as O
    nd, qi, g, po, trials = args
    rng = np.random.default_rng(11)
    worst = np.zeros(4)
    for _ in range(trials):
        q2 = qi * (1.0 + rng.choice([-1.0, 1.0], qi.shape[0]) * 2.0 ** -52)
        _, p2, _ = O.fit_segment(nd, q2, np.array(g, dtype=np.float64))
        worst = np.maximum(worst, _dist(np.asarray(p2)[None], np.asarray(po)[None])[0])
    return worst
