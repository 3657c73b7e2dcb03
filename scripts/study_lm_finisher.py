"""CPU study of the register path's literal finisher (lm.h literal_finish, in the tree of
commit 9a49333 only: it never changed a result and was reverted; profiles/r05/
lm_finisher_study.jsonl holds the output) on the random LM
vectors of tests/test_gpu_lm_stress.py: the host build of the register path with the finisher
off and on (tests/hostcheck hc_fit_segments_fin) and the literal general path, against the
C restatement (oracle/csrc/nls_scalar.c) and, for every vector any of them puts beyond 5e-10
from the C port or from each other, the numpy oracle (oracle/nls_oracle.py = the reference's
fit.fit). Prints one JSON line per ndata."""
import ctypes
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

CONSTS = np.array([100, 1e-9, 1e-9, 1e-3, 5.0, 30.0, 0.5, 0.05, 0.1, 1e-15])
LAMS = np.array([0.0, 1e-7, 1e-5, 1e-3, 1e-1, 1.0, 10.0, 100.0])


def vectors(nd, n, seed):
    from test_gpu_lm_stress import _vectors
    return _vectors(nd, n, seed)


def host(hc, qi, guess, fin_lo, fin_hi):
    n, nd2 = qi.shape
    qcm = np.ascontiguousarray(qi.T)
    p = np.zeros((n, 4))
    ssq = np.zeros(n)
    st = np.zeros(n, np.int32)
    end = np.zeros(n, np.int32)
    last = np.zeros(n)
    assert hc.hc_fit_segments_fin(qcm.ctypes.data, n, nd2 // 2, guess.ctypes.data, CONSTS.ctypes.data,
                                  LAMS.ctypes.data, 8, fin_lo, fin_hi, p.ctypes.data, ssq.ctypes.data,
                                  st.ctypes.data, end.ctypes.data, last.ctypes.data) == 0
    return st, p, ssq, end, last


def general(hc, qi, guess):
    n, nd2 = qi.shape
    qcm = np.ascontiguousarray(qi.T)
    p = np.zeros((n, 4))
    ssq = np.zeros(n)
    st = np.zeros(n, np.int32)
    hc.hc_fit_segments(qcm.ctypes.data, n, nd2 // 2, guess.ctypes.data, CONSTS.ctypes.data, LAMS.ctypes.data, 8,
                       p.ctypes.data, ssq.ctypes.data, st.ctypes.data, 1)
    return st, p, ssq


def _oracle_one(args):
    from oracle import nls_oracle as O
    nd, qi, g = args
    st, p, ssq = O.fit_segment(nd, qi, g.copy())
    return st, p


def dist(a, b):
    d = np.abs(a - b)
    d[:, 2] = np.abs((a[:, 2] - b[:, 2] + np.pi) % (2 * np.pi) - np.pi)
    return d


def main():
    hc = ctypes.CDLL(os.path.join(ROOT, "tests", "hostcheck", "libhostcheck.so"))
    P = ctypes.c_void_p
    hc.hc_fit_segments_fin.argtypes = [P, ctypes.c_long, ctypes.c_int, P, P, P, ctypes.c_int, ctypes.c_double,
                                       ctypes.c_double, P, P, P, P, P]
    hc.hc_fit_segments.argtypes = [P, ctypes.c_long, ctypes.c_int, P, P, P, ctypes.c_int, P, P, P, ctypes.c_int]
    cl = ctypes.CDLL(os.path.join(ROOT, "oracle", "libnls_scalar.so"))
    cl.lm_scalar_fit.argtypes = [P, ctypes.c_int64, ctypes.c_int, P, ctypes.c_int, P]
    from conftest import resolution_tol
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    bands = [(1e-11, 1e-8), (1e-12, 1e-7)]
    for nd in (5, 10):
        qi, guess = vectors(nd, n, 1000 + nd)
        ref = np.zeros((n, 6))
        cl.lm_scalar_fit(qi.ctypes.data, n, nd, guess.ctypes.data, 8, ref.ctypes.data)
        off = host(hc, qi, guess, 0.0, 0.0)
        ons = [host(hc, qi, guess, lo, hi) for lo, hi in bands]
        gen = general(hc, qi, guess)
        rs = ref[:, 5].astype(int)
        both0 = (rs == 0) & (off[0] == 0)
        cand = both0 & ((dist(off[1], ref[:, :4]).max(1) > 5e-10) | (dist(gen[1], ref[:, :4]).max(1) > 5e-10)
                        | np.any([dist(o[1], ref[:, :4]).max(1) > 5e-10 for o in ons], axis=0))
        idx = np.nonzero(cand)[0]
        with ProcessPoolExecutor(8) as ex:
            orc = list(ex.map(_oracle_one, [(nd, qi[k], guess[k]) for k in idx], chunksize=16))
        po = np.array([o[1] for o in orc]).reshape(-1, 4)
        tol = np.array([resolution_tol(nd, qi[k], po[i]) for i, k in enumerate(idx)]).reshape(-1, 4)

        def beyond(pp):
            return int(np.sum(np.any(dist(pp[idx], po) > tol, axis=1))) if idx.size else 0
        res = {"ndata": nd, "n": n, "status0_both": int(both0.sum()), "candidates_vs_oracle": int(idx.size),
               "beyond_resolution_vs_oracle": {"c_port": beyond(ref[:, :4]), "register": beyond(off[1]),
                                               "general": beyond(gen[1])},
               "no_lambda_end_frac": float(np.mean(off[3] & 1)),
               "last_dp_pct": [float(v) for v in np.percentile(off[4][off[3] & 1 == 1], [10, 50, 90])]}
        for (lo, hi), o in zip(bands, ons):
            res["beyond_resolution_vs_oracle"][f"register+finisher({lo:g},{hi:g})"] = beyond(o[1])
            res[f"finisher_frac({lo:g},{hi:g})"] = float(np.mean((o[3] & 2) != 0))
            res[f"status_changes({lo:g},{hi:g})"] = int(np.sum(o[0] != off[0]))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
