"""Study (numpy, CPU): the parallel-in-time EKF model of tests/test_ekf_pit_host.py on one
channel of the stress set (tests/helpers/ekf_stress.py), against the sequential EKF, for a
given sequential head T0 and block B. usage: ekf_pit_slow_channel.py BATCH CHANNEL T0 B.
Round 5: batch 0 channel 2 (m 20.9 fitted from init_m 19.4, 43 dB), a well-conditioned channel
the rule hands to the sequential kernel, needs ~29 passes with T0 = 256, ~26 with 1024 and
~24 with 2048: its error halves per pass over the whole record, not only the start-up
transient, so a longer head does not rescue it."""
import sys, numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for _p in (ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'helpers')):
    sys.path.insert(0, _p)
from test_ekf_pit_host import I5, combine, fold, identity, _ekf_step
import ekf_stress as S
bi, c, T0, B = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
n, nch, R = S.BATCHES[bi]
x, x0a, rv, qd, meta = S.batch_inputs(bi, n, nch)
x = x[c]; x0 = x0a[c]; Rv = rv[c]; q = qd
print('m %.2f snr %.1f dm %.2f'%(meta['m'][c], meta['snr_db'][c], meta['init_dm'][c]))
wt = S.W_M * (np.arange(n) / S.F_SAMP)
st, P, seq = x0.copy(), np.diag(S.P0), []
for k in range(n):
    st, P = _ekf_step(st, P, x[k], wt[k], q, Rv); seq.append(st)
seq = np.array(seq); pred = np.vstack([x0, seq[:-1]])
# when does the sequential filter lock? track m estimate
print('seq m at', [ (k, round(seq[k,1],3)) for k in (0,256,512,1024,2048,n-1)], 'true', meta['m'][c])
xbar = np.tile(x0, (n, 1))
if T0 > 0:
    xbar[:T0 + 1] = pred[:T0 + 1]; xbar[T0 + 1:] = seq[T0]
nb = (n + B - 1) // B
for it in range(30):
    aggs = []
    for b in range(nb):
        a = (np.zeros((5, 5)), x0.copy(), np.diag(S.P0), np.zeros(5), np.zeros((5, 5))) if b == 0 else identity()
        for k in range(b * B, min(n, (b + 1) * B)):
            xa, mm, ph, ps, dc = xbar[k]; th = wt[k] + ps; arg = ph + mm * np.cos(th); sa = np.sin(arg)
            h = np.array([np.cos(arg), -xa * sa * np.cos(th), -xa * sa, xa * mm * sa * np.sin(th), 1.0])
            a = fold(a, h, x[k] - (xa * np.cos(arg) + dc) + h @ xbar[k], q, Rv)
        aggs.append(a)
    pre = [aggs[0]]
    for a in aggs[1:]: pre.append(combine(pre[-1], a))
    new = np.empty_like(seq)
    for b in range(nb):
        st, P = (x0.copy(), np.diag(S.P0)) if b == 0 else (pre[b - 1][1].copy(), pre[b - 1][2].copy())
        for k in range(b * B, min(n, (b + 1) * B)):
            st, P = _ekf_step(st, P, x[k], wt[k], q, Rv); new[k] = st
    err = (np.abs(new - seq)/np.maximum(1,np.abs(seq))).max(axis=1)
    bad = np.nonzero(err > 1e-9)[0]
    print(f"pass {it+1}: max err {err.max():.2e} first bad {bad[0] if bad.size else -1} last bad {bad[-1] if bad.size else -1} nbad {bad.size}")
    xbar[1:] = new[:-1]
    if err.max() < 1e-12: break
