"""Rounding error of ssqf differences at LM minima (profiles/r04_lm_ssq_noise.txt, part 1):
ssqf(p + 1e-9 dir) - ssqf(p) by each evaluation variant of lm_ssq_variants.hip and by the
numpy oracle, against a 40-digit mpmath evaluation, at 200 config-2 minima.
Build: hipcc -O2 -std=c++17 -fPIC -shared -o $STUDY_DIR/libvar.so lm_ssq_variants.hip
Data: gen_host_study.py 0 100000 $STUDY_DIR/c2.npz"""
import sys, ctypes
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..', '..'))
import numpy as np, mpmath as mp
from oracle import nls_oracle as O
mp.mp.dps = 40
L = ctypes.CDLL(__import__('os').path.join(__import__('os').environ.get('STUDY_DIR', '/tmp/study'), 'libvar.so')); P = ctypes.c_void_p
L.var_ssq.argtypes = [P, P, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
def ssq_exact(qi, p):
    a, m, phi, psi = [mp.mpf(float(v)) for v in p]
    s = mp.mpf(0)
    for j in range(1, 11):
        c = a * mp.cos(phi + j * mp.pi / 2) * mp.besselj(j, m)
        rq = mp.mpf(float(qi[j - 1])) - c * mp.cos(j * psi); ri = mp.mpf(float(qi[j + 9])) + c * mp.sin(j * psi)
        s += rq * rq + ri * ri
    return s
z = np.load(__import__('os').path.join(__import__('os').environ.get('STUDY_DIR', '/tmp/study'), 'c2.npz')); rng = np.random.default_rng(1)
vars_ = [(0,0,0,0),(0,1,0,0),(0,3,0,0),(0,4,0,0),(0,5,0,0)]
errs = {v: [] for v in vars_}; errs['ref'] = []
for s in rng.choice(100000, 200, replace=False):
    qi = np.ascontiguousarray(z['qi'][s]); pf = z['out'][s, :4].copy()
    pts = np.ascontiguousarray(np.array([pf] + [pf + 1e-9 * rng.standard_normal(4) for _ in range(4)]))
    ex = [ssq_exact(qi, p) for p in pts]; dex = [float(e - ex[0]) for e in ex[1:]]
    for v in vars_:
        out = np.zeros(5); L.var_ssq(qi.ctypes.data, pts.ctypes.data, 5, *v, out.ctypes.data)
        errs[v] += [(out[i] - out[0]) - dex[i-1] for i in range(1, 5)]
    ref = [O.ssq_only(10, qi, p) for p in pts]
    errs['ref'] += [(ref[i] - ref[0]) - dex[i-1] for i in range(1, 5)]
for k, v in errs.items():
    v = np.array(v); print(k, 'rms %.3e max %.3e' % (np.sqrt(np.mean(v**2)), np.abs(v).max()))
