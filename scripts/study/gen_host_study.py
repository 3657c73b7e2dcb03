"""Host study data (profiles/r04_lm_ssq_noise.txt): segments [first, first+n) of the bench's
record (host restatement of the counter-based generator, oracle/philox.py), their numpy
QI (= the reference's), a phase-bin-fold QI, and the oracle's fit from the record's seed.
Usage: python gen_host_study.py FIRST N OUT.npz"""
import sys, os, time
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.abspath(__file__)), '..', '..'))
import numpy as np
from multiprocessing import Pool
from oracle import nls_oracle as O
from oracle.philox import snr_samples
from deepfmkit_amd.physics import SnrSpec
R = 4000
w0 = 2 * np.pi * 1000.0 / 200000.0
spec = SnrSpec(seed=1234, stream=0, f_samp=200000.0, f_mod=1000.0, m=6.0, snr_db=40.0)

def work(args):
    s0, n, seed = args
    x = snr_samples(spec, s0 * R, n * R).reshape(n, R)
    qi = np.array([O.demod_buffer(b, 10, w0) for b in x])
    # bin-fold QI (GPU-like summation order): bins then contraction
    t = np.arange(200)
    bas = np.array([np.cos((h + 1) * w0 * t) for h in range(10)] + [np.sin((h + 1) * w0 * t) for h in range(10)])
    bins = np.zeros((n, 200))
    for k in range(20):
        bins = bins + x[:, k * 200:(k + 1) * 200]
    qib = bins @ bas.T / R
    out = np.zeros((n, 6))
    for i in range(n):
        st, p, ssq = O.fit_segment(10, qi[i], seed.copy())
        out[i, :4] = p; out[i, 4] = ssq; out[i, 5] = st
    return qi, qib, out

if __name__ == "__main__":
    s_first, nseg = int(sys.argv[1]), int(sys.argv[2])
    x0 = snr_samples(spec, 0, R)
    _, seed, _ = O.fit_segment(10, O.demod_buffer(x0, 10, w0), np.array([1.6, 6.0, 0.0, 0.0]))
    print("seed", seed)
    step = 1000
    jobs = [(s, min(step, s_first + nseg - s), seed) for s in range(s_first, s_first + nseg, step)]
    t = time.time()
    with Pool(8) as pl:
        parts = pl.map(work, jobs)
    pl.join()
    qi = np.concatenate([p[0] for p in parts]); qib = np.concatenate([p[1] for p in parts]); out = np.concatenate([p[2] for p in parts])
    np.savez(sys.argv[3], qi=qi, qib=qib, out=out, seed=seed, first=s_first)
    print("done", time.time() - t)
