"""The LM descent modes (knob lm_spec) are schedules, not arithmetic:
- lm_spec 1, the speculative lambda ladder (lm.h lm_descend_spec): finished lanes
  evaluate later rungs of the active lanes' ladders (fit.py:221-238), and every lane
  still accepts the first improving rung in ladder order;
- lm_spec 2, one fused ssqf + coeffs evaluation per trial (lm.h FusedEval);
- lm_spec 3 (the default), the split descent with the segment's QI held in registers
  (ndata 10).
Fits must be bit-identical to the split trial / accept descent (lm_spec 0):
- the golden LM vectors (incl. noise-dominated status-2 fits, a<0 / m<0 / a=0 / m=0
  seeds, the m-grid re-seed of fit.py:336-350), every register-path ndata;
- 20k random (QI, guess) vectors from 40 dB down to noise-only, ndata 3 / 10 / 16
  (both masked register variants and the exact-ndata one): long and ragged ladders;
- whole config-2-shaped records through the fused record pipeline (rows layout) at
  40 dB and at 0 dB.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def lib():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from deepfmkit_amd import _lib
    lib = _lib.load()
    yield lib
    _lib.check(lib.dfmi_set_tuning(b"lm_spec", 3), "dfmi_set_tuning")


def _both(lib, fn):
    from deepfmkit_amd import _lib
    out = {}
    for spec in (1, 2, 0, 3):  # ends on the default
        _lib.check(lib.dfmi_set_tuning(b"lm_spec", spec), "dfmi_set_tuning")
        out[spec] = fn()
    return out


def _assert_same(r):
    for spec in (1, 2, 3):
        for x, y in zip(r[spec], r[0]):
            np.testing.assert_array_equal(np.asarray(x), np.asarray(y), err_msg=f"lm_spec {spec}")


@pytest.mark.parametrize("group", ["10", "5", "edge10"])
def test_spec_golden_vectors_bit_identical(lib, group):
    from deepfmkit_amd import fit as F
    d = np.load(os.path.join(GOLDEN, "lm_vectors.npz"))
    qi, g = d[f"g{group}_qi"], d[f"g{group}_guess"]
    nd = qi.shape[1] // 2
    r = _both(lib, lambda: F.fit_batch(nd, qi, g))
    _assert_same(r)


def _model_qi(rng, n, nd, snr_amp):
    from scipy.special import jv
    a = rng.uniform(0.5, 2.0, n)
    m = rng.uniform(0.5, 12.0, n)
    phi = rng.uniform(-np.pi, np.pi, n)
    psi = rng.uniform(-1.0, 1.0, n)
    j = np.arange(1, nd + 1)
    c = a[:, None] * np.cos(phi[:, None] + j * np.pi / 2) * jv(j, m[:, None])
    q = c * np.cos(j * psi[:, None]) + snr_amp * rng.standard_normal((n, nd))
    i = -c * np.sin(j * psi[:, None]) + snr_amp * rng.standard_normal((n, nd))
    guess = np.stack([a * rng.uniform(0.7, 1.3, n), m + rng.normal(0, 0.5, n), phi + rng.normal(0, 0.3, n),
                      psi + rng.normal(0, 0.2, n)], axis=1)
    return np.concatenate([q, i], axis=1), guess


@pytest.mark.parametrize("nd", [3, 10, 16])
def test_spec_random_vectors_bit_identical(lib, nd):
    from deepfmkit_amd import fit as F
    rng = np.random.RandomState(1000 + nd)
    parts = [_model_qi(rng, 5000, nd, s) for s in (1e-4, 1e-2, 0.3, 3.0)]
    qi = np.concatenate([p[0] for p in parts])
    g = np.concatenate([p[1] for p in parts])
    r = _both(lib, lambda: F.fit_batch(nd, qi, g))
    _assert_same(r)
    assert len(np.unique(r[0][0])) >= 2  # status 0 and the re-seeded ones both occur


@pytest.mark.parametrize("snr_noise", [0.01, 1.0])
def test_spec_record_pipeline_bit_identical(lib, snr_noise):
    import torch
    from deepfmkit_amd.fitters import nls_records
    nseg, R = 20_000, 4000
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    t = torch.arange(R, dtype=torch.float64, device="cuda") / 200000.0
    clean = 1.0 + torch.cos(6.0 * torch.cos(2 * np.pi * 1000.0 * t) + 0.3)
    x = clean.repeat(nseg) + snr_noise * torch.randn(nseg * R, dtype=torch.float64, device="cuda", generator=g)

    def run():
        cols, ok = nls_records(x.reshape(1, -1), 200000.0, 1000.0, R, nseg, 10)
        return cols.cpu().numpy(), ok.cpu().numpy()

    r = _both(lib, run)
    _assert_same(r)
