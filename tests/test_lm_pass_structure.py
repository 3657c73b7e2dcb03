"""The per-lane pass structure of the LM on config-2 segments ("LM, round
2"), counted on the oracle restatement of _run_lma_fit (fit.py:208-258): every segment
seeded from buffer 0 accepts 2 or 3 steps, and a sizeable share of lanes end with the
full 8-rung "no lambda improved" ladder (fit.py:246-247), so every 64-lane wave runs 10
one-trial passes — the fact the LM schedules of lm.h were built around."""
import numpy as np

import deepfmkit_amd as dfm
from oracle import nls_oracle as O


def test_lm_pass_structure_config2():
    R, nseg = 4000, 385
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    sim = dfm.DFMIObject("lmstats", laser, ifo, f_samp=200000.0)
    x = dfm.SignalGenerator().generate(sim, nseg * R / 200000.0, mode="snr", snr_db=40.0, trial_num=0)["main"]
    x = x.samples()
    w0 = 2 * np.pi * 1000.0 / 200000.0
    qis = [O.demod_buffer(x[s * R:(s + 1) * R], 10, w0)[:20] for s in range(nseg)]
    seed, _ = O.lm_descend(10, qis[0], [1.6, 6.0, 0.0, 0.0])
    cnt = {"trial": 0, "acc": 0}
    ssq_only, mj = O.ssq_only, O.model_and_jacobian

    def ssq_w(*a):
        cnt["trial"] += 1
        return ssq_only(*a)

    def mj_w(*a):
        cnt["acc"] += 1
        return mj(*a)

    O.ssq_only, O.model_and_jacobian = ssq_w, mj_w
    try:
        trials, accepts = [], []
        for s in range(1, nseg):
            cnt["trial"] = cnt["acc"] = 0
            O.lm_descend(10, qis[s], seed)
            trials.append(cnt["trial"])
            accepts.append(cnt["acc"] - 1)
    finally:
        O.ssq_only, O.model_and_jacobian = ssq_only, mj
    trials, accepts = np.array(trials), np.array(accepts)
    rejects = trials - accepts
    assert set(np.unique(accepts)) <= {2, 3}
    assert trials.max() == 10 and 0.05 < np.mean(rejects == 8) < 0.3
    waves = trials.reshape(-1, 64)
    assert (waves.max(axis=1) == 10).all()
    assert trials.mean() < 6.5  # the mean lane needs about half of its wave's passes
