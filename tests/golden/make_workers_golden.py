"""Golden fixtures for the trial workers (reference workers.py:132-189,
run_efficiency_trial -> run_single_trial -> DeepFitFramework.simulate(asd) + fit).
Run HERE only: imports the read-only reference (never travels to the GPU box).

Each trial: LaserConfig with f_mod = 1 kHz, df set for m_true on the default
interferometer, white amplitude noise amp_n (alpha = 0: no pyplnoise needed),
n_seconds of signal = one buffer of n = f_mod * n_seconds cycles, NLS with ndata
harmonics, init_m = m_true, parallel=False. Stored: the trial parameters and the
reference's returned m (tests/golden/workers.json).

Usage: python tests/golden/make_workers_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _import_reference  # noqa: E402

TRIALS = [dict(m_true=m, amp_n=an, n_seconds=ns, ndata=nd, trial_num=tn)
          for (m, an, ns, nd, tn) in [(6.0, 1e-4, 0.02, 10, 0), (6.0, 1e-4, 0.02, 10, 1), (4.5, 3e-4, 0.02, 10, 2),
                                      (8.0, 1e-4, 0.02, 12, 3), (12.0, 1e-4, 0.02, 16, 4), (20.0, 1e-4, 0.02, 25, 5),
                                      (6.0, 1e-3, 0.01, 10, 6), (6.0, 1e-4, 0.05, 10, 7), (9.5, 2e-4, 0.02, 14, 8),
                                      (3.0, 1e-4, 0.02, 8, 9)]]


def main():
    _import_reference()
    import DeepFMKit.physics as rphys
    import DeepFMKit.workers as rworkers
    from DeepFMKit.helpers import set_laser_df_for_effect
    out = []
    for t in TRIALS:
        laser = rphys.LaserConfig()
        laser.f_mod = 1000.0
        laser.amp_n = t["amp_n"]
        ifo = rphys.InterferometerConfig()
        set_laser_df_for_effect(laser, ifo, t["m_true"])
        params = dict(laser_config=laser, ifo_config=ifo, n_seconds=t["n_seconds"], ndata=t["ndata"],
                      m_true=t["m_true"], trial_num=t["trial_num"])
        m = rworkers.run_efficiency_trial(params)
        out.append({**t, "df": float(laser.df), "m_fit": float(m)})
        print(t, m, flush=True)
    with open(os.path.join(HERE, "workers.json"), "w") as f:
        json.dump({"trials": out, "numpy": np.__version__,
                   "source": "DeepFMKit.workers.run_efficiency_trial (workers.py:132-189)"}, f, indent=1)


if __name__ == "__main__":
    main()
