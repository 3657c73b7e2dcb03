"""Round 6: where do the short-segment (R = 200) fits beyond 1e-9 come from? The GPU study
(profiles/r06/short_parity_qi_study.jsonl) fed the device LM numpy's own QI and still got 23 of
100k beyond 1e-9: the LM's arithmetic, not the demodulation. Here the host build of lm.h
(tests/hostcheck) runs the same fits on numpy's QI of the host-generated record
(scripts/study/blas_reproducibility.py: same record, oracle fits per OpenBLAS core type) and we
count the fits beyond 1e-9 / 5e-10 of the oracle, per LM variant."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
P = ctypes.c_void_p
CONSTS = np.array([100, 1e-9, 1e-9, 1e-3, 5.0, 30.0, 0.5, 0.05, 0.1, 1e-15])
LAMS = np.array([0.0, 1e-7, 1e-5, 1e-3, 1e-1, 1.0, 10.0, 100.0])


def np_qi(X, nd, w0):
    t = np.arange(X.shape[1])
    out = np.empty((2 * nd, X.shape[0]))
    for k in range(nd):
        ang = (k + 1) * w0 * t
        c, s = np.cos(ang), np.sin(ang)
        out[k] = [(row * c).mean() for row in X]
        out[k + nd] = [(row * s).mean() for row in X]
    return out


def main():
    r, nd, nseg = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    ref = np.load(sys.argv[4])
    lib = sys.argv[5] if len(sys.argv) > 5 else os.path.join(ROOT, "tests", "hostcheck", "libhostcheck.so")
    qpath = f"/tmp/blas/qi_{r}_{nd}_{nseg}.npy"
    if os.path.exists(qpath):
        qi = np.load(qpath)
    else:
        x = np.fromfile(f"/tmp/blas/x_{r}_{nseg}.f64")
        qi = np_qi(x.reshape(nseg, r), nd, 2 * np.pi * 1000.0 / 200000.0)
        np.save(qpath, qi)
    hc = ctypes.CDLL(lib)
    hc.hc_fit_segments.argtypes = [P, ctypes.c_long, ctypes.c_int, P, P, P, ctypes.c_int, P, P, P, ctypes.c_int]
    n1 = nseg - 1
    q1 = np.ascontiguousarray(qi[:, 1:])
    guess = np.ascontiguousarray(np.tile(ref[0, :4], (n1, 1)))
    ok = ref[1:, 6] == 0
    for fg in [int(v) for v in (sys.argv[6].split(",") if len(sys.argv) > 6 else ["0", "1"])]:
        gp = np.zeros((n1, 4)); ss = np.zeros(n1); gs = np.zeros(n1, np.int32)
        hc.hc_fit_segments(q1.ctypes.data, n1, nd, guess.ctypes.data, CONSTS.ctypes.data, LAMS.ctypes.data, 8,
                           gp.ctypes.data, ss.ctypes.data, gs.ctypes.data, fg)
        d = np.abs(gp - ref[1:, :4])
        d[:, 2] = np.abs((gp[:, 2] - ref[1:, 2] + np.pi) % (2 * np.pi) - np.pi)
        d[~ok] = 0
        dm = d.max(axis=1)
        bad = np.nonzero(dm > 1e-9)[0] + 1
        print(f"force_general={fg}: status mismatch {int(np.sum(gs != ref[1:, 6]))}, identical {int(np.sum(dm == 0))}, "
              f">5e-10 {int(np.sum(dm > 5e-10))}, >1e-9 {bad.size}, max {d.max(axis=0).tolist()} bad {bad[:30].tolist()}")


if __name__ == "__main__":
    main()
