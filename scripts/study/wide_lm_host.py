"""Round 6: the many-harmonic LM path (lm.h kWideNd) on the host build (tests/hostcheck,
force_general = 3) against the numpy oracle, before any GPU run: the golden LM vectors of
ndata 20 / 30 / 62 (tests/golden/lm_vectors.npz, from the reference) and config-2-like
segments (host philox record, numpy QI) at ndata 20 / 30 / 62, m 6 and 31.4."""
import ctypes
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
P = ctypes.c_void_p
CONSTS = np.array([100, 1e-9, 1e-9, 1e-3, 5.0, 30.0, 0.5, 0.05, 0.1, 1e-15])
LAMS = np.array([0.0, 1e-7, 1e-5, 1e-3, 1e-1, 1.0, 10.0, 100.0])


def hc_fit(qi_rows, guess, nd, mode):
    hc = ctypes.CDLL(os.path.join(ROOT, "tests", "hostcheck", "libhostcheck.so"))
    hc.hc_fit_segments.argtypes = [P, ctypes.c_long, ctypes.c_int, P, P, P, ctypes.c_int, P, P, P, ctypes.c_int]
    n = qi_rows.shape[0]
    q = np.ascontiguousarray(qi_rows.T)
    g = np.ascontiguousarray(guess)
    gp = np.zeros((n, 4)); ss = np.zeros(n); gs = np.zeros(n, np.int32)
    hc.hc_fit_segments(q.ctypes.data, n, nd, g.ctypes.data, CONSTS.ctypes.data, LAMS.ctypes.data, 8, gp.ctypes.data,
                       ss.ctypes.data, gs.ctypes.data, mode)
    return gs, gp, ss


def ofit(args):
    from oracle import nls_oracle as O
    nd, qi, g = args
    st, p, ssq = O.fit_segment(nd, qi, np.array(g))
    return st, p, ssq


def dist(a, b):
    d = np.abs(a - b)
    d[:, 2] = np.abs((a[:, 2] - b[:, 2] + np.pi) % (2 * np.pi) - np.pi)
    return d


def report(name, nd, qi, guess, st_r, p_r, ss_r):
    for mode in (1, 3):
        gs, gp, ss = hc_fit(qi, guess, nd, mode)
        ok = (st_r == 0) & (gs == 0)
        d = dist(gp, p_r)[ok]
        rel = np.abs(ss - ss_r)[ok] / np.maximum(ss_r[ok], 1e-300)
        print(f"{name} nd={nd} mode={'literal' if mode == 1 else 'wide'}: status mismatch {int(np.sum(gs != st_r))}"
              f"/{len(st_r)}, max |d| {d.max(axis=0) if d.size else 0}, >1e-9 {int(np.sum(d.max(axis=1) > 1e-9))}, "
              f"ssq rel {rel.max() if rel.size else 0:.2e}", flush=True)


def main():
    lm = np.load(os.path.join(ROOT, "tests", "golden", "lm_vectors.npz"))
    for grp in ("20", "30", "62"):
        qi, g = lm[f"g{grp}_qi"], lm[f"g{grp}_guess"]
        report(f"golden g{grp}", qi.shape[1] // 2, qi, g, lm[f"g{grp}_status"], lm[f"g{grp}_p"], lm[f"g{grp}_ssq"])
    from deepfmkit_amd.physics import SnrSpec
    from oracle import philox
    from oracle import nls_oracle as O
    nseg, R = int(os.environ.get("NSEG", 3000)), 4000
    w0 = 2 * np.pi * 1000.0 / 200000.0
    for m in (6.0, 31.4):
        spec = SnrSpec(seed=1234, stream=0, f_samp=200000.0, f_mod=1000.0, m=m, snr_db=40.0)
        x = philox.snr_samples(spec, 0, nseg * R).reshape(nseg, R)
        for nd in (20, 30, 62):
            qi = np.stack([O.demod_buffer(x[i], nd, w0) for i in range(nseg)])
            st0, p0, _ = ofit((nd, qi[0], [1.6, 6.0, 0.0, 0.0]))
            guess = np.tile(p0, (nseg - 1, 1))
            with ProcessPoolExecutor(8) as ex:
                res = list(ex.map(ofit, [(nd, qi[i], p0) for i in range(1, nseg)], chunksize=64))
            report(f"record m={m}", nd, qi[1:], guess, np.array([r[0] for r in res]), np.stack([r[1] for r in res]),
                   np.array([r[2] for r in res]))


if __name__ == "__main__":
    main()
