"""The GPU LM (dfmi_lm: fit.fit, fit.py:322-361, every vector its own guess) on 600,000
random QI vectors, screened against the scalar C restatement of fit.fit (oracle/csrc/nls_scalar.c
lm_scalar_fit) and judged against the numpy oracle itself (oracle/nls_oracle.py = the
reference's fit.fit, bit-exact on its golden vectors), as a stress test across the parameter
space the golden vectors sample only sparsely: ndata 5 / 10 / 16 (exact-ndata register path,
masked register path, and the 16-harmonic variant), amplitude 0.2..3, m 1..25, any phi, psi in
[-1, 1], noise from 1e-7 to 1e-1 of the amplitude, guesses from near the truth to far off
(m-grid re-seeds, status 1 / 2, sign normalisation, phi wrap).

Gates: status equal to the C port's on >= 99.9 % of the vectors. Where both report status 0,
every vector the GPU puts more than 5e-10 from the C port is refitted by the numpy oracle;
it must be within max(1e-9, the reference's resolution, conftest.resolution_tol) of the
oracle's answer, or within 1.5x the oracle's OWN move when its QI moves by one ulp
(tests/helpers/lm_oracle_check.py: there the reference's answer is set by its last bits, not
by its algorithm). At most 1e-4 of the status-0 vectors may miss both (measured round 5 on
the host build of the same arithmetic: the register path beyond the resolution on 35 of
160,906 ndata-5 vectors, the literal C port on 25, the literal general path on 40; a literal
"finisher" of the register path changed none of them, profiles/r05/lm_finisher_study.jsonl)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import wrapped

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
    cand = np.nonzero(both0 & (d.max(axis=1) > 5e-10))[0]
    import multiprocessing as mp
    import sys
    from concurrent.futures import ProcessPoolExecutor
    sys.path.insert(0, os.path.join(ROOT, "tests", "helpers"))
    import lm_oracle_check as LC
    procs = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 8))
    with ProcessPoolExecutor(procs, mp_context=mp.get_context("spawn")) as ex:
        orc = list(ex.map(LC.oracle_fit, [(nd, qi[k], guess[k]) for k in cand], chunksize=32))
        beyond = [(k, o) for k, o in zip(cand, orc) if o[0] == 0 and np.any(LC._dist(gp[k][None], o[1][None])[0] > o[2])]
        spreads = list(ex.map(LC.oracle_spread, [(nd, qi[k], guess[k], o[1], 4) for k, o in beyond]))
    unexplained = [int(k) for (k, o), sp in zip(beyond, spreads)
                   if np.any(LC._dist(gp[k][None], o[1][None])[0] > np.maximum(o[2], 1.5 * sp))]
    n0 = max(1, int(both0.sum()))
    print(f"ndata {nd}: status match {match.mean():.5f}, status-0 {both0.mean():.3f}, beyond 5e-10 of the C port "
          f"{cand.size}, beyond the resolution of the numpy oracle {len(beyond)}, of those beyond the oracle's own "
          f"one-ulp spread {len(unexplained)} ({len(unexplained) / n0:.2e})")
    assert len(unexplained) <= 1e-4 * n0, unexplained[:10]
