"""The oracle's LM decisions on given segments (profiles/r04_lm_ssq_noise.txt, part 2).
Usage: python trace_oracle_lm.py c4.npz 1249633 ..."""
import sys
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..', '..'))
import numpy as np
from oracle import nls_oracle as O
z = np.load(sys.argv[1]); first = int(z['first'])
for s in map(int, sys.argv[2:]):
    qi = z['qi'][s - first]; p = z['seed'].copy()
    ssq0, jtj, g = O.model_and_jacobian(10, qi, p)
    print('seg', s, 'ssq0', ssq0)
    for it in range(100):
        pp = p.copy(); found = False
        for lam in O.LAMBDA_LADDER:
            dp = O.damped_step(lam, jtj, g)
            if np.linalg.norm(dp) < 1e-15: print('   skip lam', lam); continue
            tr = p + dp; s_ = O.ssq_only(10, qi, tr)
            print(f'  it{it} lam {lam:g} |dp| {np.linalg.norm(dp):.3e} ssq_try-ssq0 {s_-ssq0:.3e} ({(s_-ssq0)/np.spacing(ssq0):.1f} ulp)', 'ACC' if s_ < ssq0 else 'rej')
            if s_ < ssq0: found = True; best = s_; p = tr; break
        if not found: print('  no lambda'); break
        ssq0, jtj, g = O.model_and_jacobian(10, qi, p)
        if ssq0 - best < 1e-9 and np.linalg.norm(p - pp) < 1e-9: print('  converged'); break
    w, v = np.linalg.eigh(jtj.reshape(4,4)); print('  JtJ eig', w, 'ssq', ssq0)
