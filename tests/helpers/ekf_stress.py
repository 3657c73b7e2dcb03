"""Randomised channels for the EKF parallel-in-time stress test (tests/test_gpu_ekf_pit_stress.py,
scripts/probe_pit_rule.py) and the scalar C oracle they are checked against
(oracle/csrc/ekf_scalar.c: EKFFitter.fit's loop, fitters.py:274-307, in numpy's operation order).

Each batch is one dfmi_ekf call (EKFFitter.fit with the caller's x0 and R_val,
fitters.py:241-257): channels of one length and one Q_diag, each with its own record, x0
(init_a / init_m / init_phi / init_psi offsets, dc = np.mean) and R_val (np.var scaled).
Signals: the snr-mode model a (1 + C cos(phi + m cos(w_m t + psi))) + white noise
(physics.py:475-530's formula, numpy Generator noise: the draws need not match the
reference's — both sides of the comparison read the same array)."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
F_SAMP, F_MOD = 200000.0, 1000.0
W_M = 2 * np.pi * F_MOD
P0 = np.ones(5)
QD0 = np.array([1e-8, 1e-8, 1e-6, 1e-6, 1e-8])

# (length, channels, R) per batch: 4,096 .. 400,000 samples, >= 500 channels in all,
# ~55 M samples for the scalar oracle (~6 s on one host core)
BATCHES = [(4096, 96, 1024), (4096, 32, 4000), (10000, 96, 2000), (25000, 64, 4000), (40003, 64, 3000),
           (100000, 64, 4000), (100000, 32, 7), (200000, 32, 4000), (400000, 24, 4000)]


def batch_inputs(bi, length, nch, seed=2025):
    """Records (nch, length), x0 (nch, 5), r_val (nch,), q_diag (5,) of batch bi."""
    rng = np.random.default_rng([seed, bi])
    t = np.arange(length) / F_SAMP
    m = rng.uniform(1.0, 25.0, nch)
    phi = rng.uniform(-np.pi, np.pi, nch)
    psi = rng.uniform(-np.pi, np.pi, nch)
    amp = rng.uniform(0.5, 2.0, nch)
    vis = rng.uniform(0.3, 1.0, nch)
    snr_db = rng.uniform(0.0, 60.0, nch)
    x = np.empty((nch, length))
    for c in range(nch):
        clean = amp[c] * (1.0 + vis[c] * np.cos(phi[c] + m[c] * np.cos(W_M * t + psi[c])))
        ac = amp[c] * vis[c]
        noise_std = ac / np.sqrt(2.0) / 10 ** (snr_db[c] / 20.0)
        x[c] = clean + rng.normal(0.0, noise_std, length)
    x0 = np.empty((nch, 5))
    x0[:, 0] = amp * vis * rng.uniform(0.5, 1.5, nch)
    x0[:, 1] = np.maximum(m + rng.uniform(-4.0, 4.0, nch), 0.1)
    x0[:, 2] = phi + rng.uniform(-1.0, 1.0, nch)
    x0[:, 3] = psi + rng.uniform(-0.5, 0.5, nch)
    x0[:, 4] = x.mean(axis=1)
    r_val = x.var(axis=1) * 10 ** rng.uniform(-2.0, 2.0, nch)
    qd = QD0 * 10 ** rng.uniform(-2.0, 2.0)
    meta = {"m": m, "phi": phi, "psi": psi, "snr_db": snr_db, "init_dm": x0[:, 1] - m}
    return np.ascontiguousarray(x), np.ascontiguousarray(x0), np.ascontiguousarray(r_val), qd, meta


def c_oracle():
    so = os.path.join(ROOT, "oracle", "libekf_scalar.so")
    if not os.path.exists(so):
        return None
    cl = ctypes.CDLL(so)
    P = ctypes.c_void_p
    cl.ekf_scalar.argtypes = [P, ctypes.c_int64, P, P, P, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                              ctypes.c_int64, ctypes.c_int64, P]
    return cl


def c_states(cl, x, x0, r_val, qd, R, nbuf):
    st = np.zeros((nbuf, 5))
    x = np.ascontiguousarray(x)
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    q = np.ascontiguousarray(qd, dtype=np.float64)
    cl.ekf_scalar(x.ctypes.data, x.size, x0.ctypes.data, P0.ctypes.data, q.ctypes.data, float(r_val), W_M, F_SAMP, R,
                  nbuf, st.ctypes.data)
    return st


def gpu_states(lib, x, x0, r_val, qd, R, nbuf):
    """dfmi_ekf over the batch (host memory): states (nch, nbuf, 5), kernel name, passes."""
    from deepfmkit_amd import _lib
    nch, n = x.shape
    st = np.zeros((nch, nbuf, 5))
    q = np.ascontiguousarray(qd, dtype=np.float64)
    _lib.check(lib.dfmi_ekf(_lib.ptr(x), nch, n, n, _lib.ptr(x0), _lib.ptr(P0), _lib.ptr(q), _lib.ptr(r_val), W_M,
                            F_SAMP, R, nbuf, _lib.ptr(st), _lib.DFMI_MEM_HOST, None), "dfmi_ekf")
    kname = lib.dfmi_last_demod_kernel().decode()
    passes = (ctypes.c_int32 * nch)()
    _lib.check(lib.dfmi_ekf_pit_passes(ctypes.cast(passes, ctypes.c_void_p), nch), "passes")
    return st, kname, np.array(list(passes))


def rel_err(got, ref):
    """Largest |got - ref| / max(1, |ref|) per channel (the stop rule's own measure)."""
    return (np.abs(got - ref) / np.maximum(1.0, np.abs(ref))).reshape(got.shape[0], -1).max(axis=1)


def sensitivity(cl, x, x0, r_val, qd, R, nbuf, ref=None):
    """How far the oracle's own states move under rounding-sized perturbations: the C loop
    rerun with every sample scaled by (1 +- 2^-52) (signs from a fixed generator) and with x0
    scaled by (1 + 1e-15); the larger relative move over the snapshots. A well-conditioned
    channel moves ~1e-15; a filter that has not locked is chaotic and moves by up to O(1) —
    there no two correct implementations (GPU or CPU, numpy's or libm's rounding) agree to
    1e-12, and the gate scales with this number (tests/test_gpu_ekf_pit_stress.py)."""
    if ref is None:
        ref = c_states(cl, x, x0, r_val, qd, R, nbuf)
    sg = np.where(np.random.default_rng(7).random(x.size) < 0.5, -1.0, 1.0)
    xp = x * (1.0 + sg * 2.0 ** -52)
    s1 = c_states(cl, xp, x0, r_val, qd, R, nbuf)
    s2 = c_states(cl, x, x0 * (1.0 + 1e-15), r_val, qd, R, nbuf)
    return float(max(rel_err(s1[None], ref[None])[0], rel_err(s2[None], ref[None])[0]))


def oracle_batch(cl, x, x0, r_val, qd, R, nbuf, threads=8):
    """Oracle states (nch, nbuf, 5) and sensitivities (nch,) of a batch, channels in parallel
    threads (the ctypes call releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor

    def one(c):
        ref = c_states(cl, x[c], x0[c], r_val[c], qd, R, nbuf)
        return ref, sensitivity(cl, x[c], x0[c], r_val[c], qd, R, nbuf, ref=ref)
    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(one, range(x.shape[0])))
    return np.stack([r[0] for r in res]), np.array([r[1] for r in res])
