"""The W-DFMI oracle (oracle/wdfmi_oracle.py) pinned to the reference's own outputs.

tests/golden/wdfmi.npz holds inputs and outputs of WDFMI_NLSFitter,
WDFMI_OrthogonalFitter, WDFMI_SequentialFitter and HWDFMI_Fitter
(fitters.py:481-891) run by tests/golden/make_wdfmi_golden.py. The oracle restates
scipy's Nelder-Mead / bracket / Brent / bounded-Brent and MINPACK lmdif in plain
Python; on these fixtures it reproduces the reference bit for bit.
"""
import json
import os

import numpy as np
import pytest

from oracle import wdfmi_oracle as W

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "wdfmi.npz"))
CASES = {c["name"]: c for c in json.load(open(os.path.join(HERE, "golden", "wdfmi_cases.json")))["cases"]}
COLS = ["amp", "m", "phi", "psi", "tau", "dc", "ssq", "fitok"]


def run_oracle(case, method, main=None):
    f_samp, f_mod, df, meas, ref, f_ref, n = G[f"{case}_cfg"]
    c = CASES[case]
    main = G[f"{case}_main"] if main is None else main
    wit = G[f"{case}_witness"]
    dl, n = meas - ref, int(n)
    if method == "wdfmi_nls":
        return W.fit_wdfmi_nls(main, wit, f_samp, f_mod, df, dl, n, **c["nls"])
    if method == "wdfmi_ortho":
        return W.fit_wdfmi_ortho(main, wit, f_samp, f_mod, df, dl, n, **c["ortho"])
    if method == "wdfmi_seq":
        return W.fit_wdfmi_seq(main, wit, f_samp, f_mod, df, dl, n, **c["seq"])
    return W.fit_hwdfmi(main, G[f"{case}_hw_witness"], f_samp, f_mod, f_ref, dl, n)


@pytest.mark.parametrize("case", ["cos", "dist"])
@pytest.mark.parametrize("method", ["wdfmi_nls", "wdfmi_ortho", "wdfmi_seq", "hwdfmi"])
def test_oracle_matches_reference_bit_exact(case, method):
    out = run_oracle(case, method)
    for k in COLS:
        np.testing.assert_array_equal(out[k], G[f"{case}_{method}_{k}"], err_msg=f"{case} {method} {k}")


def test_minpack_restatement_known_problem():
    """lmdif on a textbook problem (Rosenbrock as residuals) reaches the minimum."""
    x, f, info = W.lmdif(lambda p: np.array([10 * (p[1] - p[0] ** 2), 1 - p[0]]), [-1.2, 1.0])
    assert info in (1, 2, 3, 4)
    np.testing.assert_allclose(x, [1.0, 1.0], atol=1e-7)


def test_scalar_minimisers_known_answers():
    x, fx, ok = W.brent(lambda u: (u - 0.3) ** 2 + 1.0, (0.0, 1.0))
    assert ok and abs(x - 0.3) < 1e-7
    x, fx, flag = W.fminbound(lambda u: np.cos(u), 2.0, 4.0)
    assert flag == 0 and abs(x - np.pi) < 1e-4
    x, fx, ok = W.nelder_mead(lambda p: (p[0] - 1) ** 2 + (p[1] + 2) ** 2, [0.0, 0.0])
    assert ok and np.allclose(x, [1, -2], atol=1e-3)


def test_reference_sensitivity():
    """How finely the reference determines its own answer (sets the GPU tolerances in
    tests/test_gpu_wdfmi.py): perturb the main channel by ~1 ulp (relative 2e-16) and
    re-run the restated reference. ortho / hwdfmi follow the same optimiser path (tau,
    psi move by at most an ulp); seq's psi stage moves by ~1e-7; nls on the distorted
    case is chaotic (tens of percent)."""
    rng = np.random.default_rng(1)

    def spread(case, method):
        a = run_oracle(case, method)
        main = G[f"{case}_main"]
        b = run_oracle(case, method, main=main * (1 + rng.standard_normal(main.shape) * 2e-16))
        return {k: float(np.max(np.abs(a[k] - b[k]) / np.abs(a[k]))) for k in ("amp", "phi", "psi", "tau")}

    s = spread("cos", "wdfmi_ortho")
    assert s["tau"] <= 1e-15 and s["psi"] <= 1e-15 and s["amp"] < 1e-14
    s = spread("cos", "hwdfmi")
    assert s["tau"] <= 1e-15 and s["amp"] < 1e-14
    s = spread("cos", "wdfmi_seq")
    assert 1e-9 < s["psi"] < 1e-5
    s = spread("dist", "wdfmi_nls")
    assert s["amp"] > 1e-3
