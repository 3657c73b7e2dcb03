"""The GPU LM (dfmi_lm: fit.fit, fit.py:322-361, every vector its own guess) on 600,000
random QI vectors against the scalar C restatement of fit.fit (oracle/csrc/nls_scalar.c
lm_scalar_fit, which meets the reference's own LM vectors with the GPU's gates:
tests/test_oracle_c.py), as a stress test across the parameter space the golden vectors
sample only sparsely: ndata 5 / 10 / 16 (exact-ndata register path, masked register path,
and the 16-harmonic variant), amplitude 0.2..3, m 1..25, any phi, psi in [-1, 1], noise from
1e-7 to 1e-1 of the amplitude, guesses from near the truth to far off (m-grid re-seeds,
status 1 / 2, sign normalisation, phi wrap).

Gates: status equal on >= 99.9 % of the vectors; where both report status 0, every
parameter within max(1e-9, the reference's resolution, conftest.resolution_tol) on
>= 99.9 % of them. Measured (profiles/r03q_lm_stress.log): status equal on all 600,000;
beyond the resolution 79 / 161 k (ndata 5), 16 / 146 k (10), 14 / 139 k (16). Those are
ill-conditioned, low-noise fits where the LM ends on "no lambda improved" about 1e-9 from
the minimum, at a point set by the last bits of the Jacobian and of ssq: on 40 such ndata-5
vectors the host build of the register path lands beyond the resolution from the numpy
oracle (= the reference) on 31, and the literal C restatement itself on 7 — the
reference's answer there is not determined to 1e-9 by its algorithm, only by its exact
arithmetic (cos(fl(phi + j pi/2)), scipy's jv, BLAS summation order)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import resolution_tol, wrapped

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _vectors(nd, n, seed):
    from scipy.special import jv
    rng = np.random.default_rng(seed)
    a = rng.uniform(0.2, 3.0, n)
    m = rng.uniform(1.0, 25.0, n)
    phi = rng.uniform(-np.pi, np.pi, n)
    psi = rng.uniform(-1.0, 1.0, n)
    j = np.arange(1, nd + 1)
    common = a[:, None] * np.cos(phi[:, None] + j * np.pi / 2.0) * jv(j, m[:, None])
    q = common * np.cos(j * psi[:, None])
    i = -common * np.sin(j * psi[:, None])
    noise = a * 10.0 ** rng.uniform(-7, -1, n)
    qi = np.concatenate([q, i], axis=1) + noise[:, None] * rng.standard_normal((n, 2 * nd))
    far = rng.uniform(0, 1, n) < 0.2
    spread = np.where(far, 1.0, 1e-2)
    guess = np.stack([a * (1 + spread * rng.uniform(-0.5, 0.5, n)), m * (1 + spread * rng.uniform(-0.3, 0.3, n)),
                      phi + spread * rng.uniform(-1, 1, n), psi + spread * rng.uniform(-0.3, 0.3, n)], axis=1)
    return np.ascontiguousarray(qi), np.ascontiguousarray(guess)


@pytest.mark.parametrize("nd", [5, 10, 16])
def test_gpu_lm_random_vectors_vs_c_restatement(nd):
    import torch
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    so = os.path.join(ROOT, "oracle", "libnls_scalar.so")
    if not os.path.exists(so):
        pytest.skip("oracle/libnls_scalar.so not built")
    n = 200_000
    qi, guess = _vectors(nd, n, 1000 + nd)
    cl = ctypes.CDLL(so)
    P = ctypes.c_void_p
    cl.lm_scalar_fit.argtypes = [P, ctypes.c_int64, ctypes.c_int, P, ctypes.c_int, P]
    ref = np.zeros((n, 6))
    assert cl.lm_scalar_fit(qi.ctypes.data, n, nd, guess.ctypes.data, min(16, os.cpu_count() or 1),
                            ref.ctypes.data) == 0
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    qd = torch.from_numpy(np.ascontiguousarray(qi.T)).to(dev)
    gd = torch.from_numpy(guess).to(dev)
    p = torch.empty((4, n), dtype=torch.float64, device=dev)
    ssq = torch.empty(n, dtype=torch.float64, device=dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    _lib.check(lib.dfmi_lm(qd.data_ptr(), n, nd, gd.data_ptr(), 1, n, F.lm_config(), p.data_ptr(), ssq.data_ptr(),
                           st.data_ptr(), _lib.DFMI_MEM_DEVICE, torch.cuda.current_stream().cuda_stream), "dfmi_lm")
    torch.cuda.synchronize()
    gp, gs = p.cpu().numpy().T, st.cpu().numpy()
    rs = ref[:, 5].astype(int)
    match = gs == rs
    assert match.mean() >= 0.999, (match.mean(), np.bincount(rs), np.bincount(gs))
    both0 = match & (rs == 0)
    d = np.stack([np.abs(gp[:, 0] - ref[:, 0]), np.abs(gp[:, 1] - ref[:, 1]), wrapped(gp[:, 2] - ref[:, 2]),
                  np.abs(gp[:, 3] - ref[:, 3])], axis=1)
    cand = np.nonzero(both0 & (d.max(axis=1) > 1e-9))[0]
    bad = [int(k) for k in cand if np.any(d[k] > resolution_tol(nd, qi[k], ref[k, :4]))]
    frac_bad = len(bad) / max(1, int(both0.sum()))
    print(f"ndata {nd}: status match {match.mean():.5f}, status-0 {both0.mean():.3f}, beyond 1e-9 {cand.size}, "
          f"beyond resolution {len(bad)}")
    assert frac_bad <= 1e-3, (len(bad), bad[:5], d[bad[:5]] if bad else None)
