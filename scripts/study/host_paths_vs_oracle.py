"""Host builds of the LM paths (tests/hostcheck) against the oracle on study data
(profiles/r04_lm_ssq_noise.txt, part 3). Usage: python host_paths_vs_oracle.py c2.npz c4.npz"""
import sys, ctypes
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..', '..')); sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..', '..', 'tests'))
import numpy as np
hc = ctypes.CDLL(__import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..', '..', 'tests', 'hostcheck', 'libhostcheck.so'))
P = ctypes.c_void_p
hc.hc_fit_segments.argtypes = [P, ctypes.c_long, ctypes.c_int, P, P, P, ctypes.c_int, P, P, P, ctypes.c_int]
def fit(qi, seed, fg):
    n = qi.shape[0]
    consts = np.array([100, 1e-9, 1e-9, 1e-3, 5.0, 30.0, 0.5, 0.05, 0.1, 1e-15])
    lams = np.array([0.0, 1e-7, 1e-5, 1e-3, 1e-1, 1.0, 10.0, 100.0])
    qcm = np.ascontiguousarray(qi.T); g = np.ascontiguousarray(np.tile(seed, (n, 1)))
    p = np.zeros((n, 4)); ssq = np.zeros(n); st = np.zeros(n, np.int32)
    hc.hc_fit_segments(qcm.ctypes.data, n, 10, g.ctypes.data, consts.ctypes.data, lams.ctypes.data, 8, p.ctypes.data, ssq.ctypes.data, st.ctypes.data, fg)
    return p, st
def dev(p, ref):
    d = np.abs(p - ref[:, :4]); d[:, 2] = np.abs((p[:, 2] - ref[:, 2] + np.pi) % (2 * np.pi) - np.pi)
    return d.max(1)
for f in sys.argv[1:]:
    z = np.load(f); ref = z['out']; seed = z['seed']
    print(f, 'status counts', np.bincount(ref[:, 5].astype(int)))
    for qn in ('qi', 'qib'):
        for fg in (0, 1):
            p, st = fit(z[qn], seed, fg)
            d = dev(p, ref); d[st != ref[:, 5]] = 0
            o = np.argsort(d)[::-1][:5]
            print(f"  {qn} general={fg} max {d.max():.3e} >3e-10 {np.sum(d>3e-10)} >5e-10 {np.sum(d>5e-10)} >1e-9 {np.sum(d>1e-9)} status mismatch {np.sum(st != ref[:,5])} worst {o + z['first']} {d[o]}")
