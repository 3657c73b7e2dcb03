"""§8f-2 (second half): Experiment.run batched on the GPU (deepfmkit_amd/experiments.py)
vs the reference's per-trial Pool path restated on the CPU.

Workload: notebooks/5.0_Experiment.ipynb's sweep — VairableAmplitudeOffset factory
(m_main = 5, nominal_amplitude axis of 10 points, a stochastic amplitude offset with
5 % relative std, default 10 fit buffers = one 2000-sample record per trial fitted as
one n = 10 buffer) with an NLS analysis (ndata = 10) — scaled to TRIALS trials per
point. Reported: end-to-end trials/s of Experiment.run (job list + factory calls +
device synthesis + one batched fit + aggregation), the device-resident phases, and a
CPU baseline: the same trials through the reference's per-trial worker restated on one
core (host simulation + the oracle's single-buffer fit), on a sample.
"""
import json
import os
import sys
import time
from functools import partial

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def offset_gen(nominal_amplitude, relative_noise_std):
    return np.random.normal(loc=0.0, scale=nominal_amplitude * relative_noise_std)


def build(trials_per_point):
    from deepfmkit_amd.experiments import Experiment
    from deepfmkit_amd.factories import VairableAmplitudeOffset
    exp = Experiment("notebook 5.0 sweep")
    exp.set_config_factory(VairableAmplitudeOffset(opd_main=0.1))
    exp.add_axis("nominal_amplitude", np.linspace(0.5, 2.0, 10))
    exp.set_static({"m_main": 5.0})
    exp.add_stochastic_variable("amplitude_offset", partial(offset_gen, relative_noise_std=0.05),
                                depends_on="nominal_amplitude")
    exp.n_trials = trials_per_point
    exp.add_analysis("NLS_Fit", "nls", result_cols=["amp", "m", "phi", "psi", "ssq"],
                     fitter_kwargs={"n": 20, "ndata": 10})
    return exp


def main():
    import torch

    from deepfmkit_amd import experiments as E
    from deepfmkit_amd import physics as P
    from oracle import nls_oracle as O

    tpp = int(os.environ.get("TRIALS", 1000))
    warm = build(4)
    np.random.seed(0)
    warm.run()
    torch.cuda.synchronize()
    out = {"metric": "Experiment.run trials/s (notebook 5.0 sweep: 10 points, NLS, one 2000-sample buffer per trial)"}
    for n in sorted({100, tpp}):
        exp = build(n)
        np.random.seed(0)
        t0 = time.perf_counter()
        res = exp.run()
        el = time.perf_counter() - t0
        out[f"trials_{10 * n}"] = {"seconds": round(el, 4), "trials_per_s": round(10 * n / el, 1),
                                   "amp_mean": [round(float(v), 6) for v in res["NLS_Fit"]["amp"]["mean"]]}
    # device-resident phases of the largest run: synthesis + the one fit call
    exp = build(tpp)
    np.random.seed(0)
    trials = [E._Trial(p, k, exp.config_factory(p), exp.n_fit_buffers_per_trial, exp.f_samp)
              for p, k in exp._job_list()]
    E._synthesize(trials)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record(st)
    E._synthesize(trials)
    ev[1].record(st)
    E._fit_batched(trials, exp.analyses[0], exp.n_fit_buffers_per_trial)
    ev[2].record(st)
    torch.cuda.synchronize()
    out["device_phases_ms"] = {"synthesis": round(ev[0].elapsed_time(ev[1]), 3),
                               "fit_and_means": round(ev[1].elapsed_time(ev[2]), 3)}
    # CPU baseline: the reference's worker per trial, restated (1 core), on a sample
    nb = int(os.environ.get("CPU_TRIALS", 100))
    t0 = time.perf_counter()
    dm = 0.0
    res_gpu = E._fit_batched(trials[:nb], exp.analyses[0], exp.n_fit_buffers_per_trial)
    t0 = time.perf_counter()
    for k, t in enumerate(trials[:nb]):
        x = np.asarray(P.SignalGenerator().generate(t.main, t.n_seconds, mode="asd", trial_num=t.num)["main"]
                       .samples())
        R = int(t.f_samp / t.main.laser.f_mod * exp.n_fit_buffers_per_trial)
        r = O.fit_chunk((x.reshape(-1, R), np.array([1.6, 6.0, 0.0, 0.0]), 10, t.main.laser.f_mod, t.f_samp,
                         dict(O.C0)))
        dm = max(dm, abs(r[0][1] - res_gpu[k]["m"]))
    cpu = nb / (time.perf_counter() - t0)
    out["cpu_baseline"] = {"value": round(cpu, 1), "unit": "trials/s", "cores": 1, "kind": "port",
                           "sample": f"{nb} trials: host asd simulation + oracle single-buffer fit per trial"}
    out["max_abs_dm_gpu_vs_oracle"] = dm
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
