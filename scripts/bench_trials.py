"""§8f-2: trial batching for the experiment workers (workers.py:132-189). Many
efficiency trials (one buffer each: m_true = 6, white amplitude noise 1e-4, 20 ms at
200 kS/s = one R = 4000 buffer, ndata = 10) through workers.run_efficiency_trials:
records generated on the GPU (dfmi_synth_asd: numpy's RandomState stream and the
asd-mode exact-delay model, one lane per trial) and fitted as records of ONE GPU
call, vs the reference's one-trial-per-call loop restated on the CPU (the package's
host simulation + the oracle's single-buffer fit, 1 core).

Reported: end-to-end trials/s of the batched worker (Python set-up + device synthesis
+ fit + m back on the host), the same with the host generator (synth="host", on a
sample), the synthesis call (host set-up of the trial table + upload + kernel) and the
fit alone (HIP events, records resident),
and the CPU baseline."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import deepfmkit_amd as dfm
    from deepfmkit_amd import fitters as F
    from deepfmkit_amd import physics as P
    from deepfmkit_amd import workers
    from oracle import nls_oracle as O

    ntr = int(os.environ.get("TRIALS", 20000))
    nhost = int(os.environ.get("HOST_TRIALS", 2000))

    def params(i):
        laser = dfm.LaserConfig()
        laser.f_mod = 1000.0
        laser.amp_n = 1e-4
        ifo = dfm.InterferometerConfig()
        dfm.set_laser_df_for_effect(laser, ifo, 6.0)
        return dict(laser_config=laser, ifo_config=ifo, n_seconds=0.02, ndata=10, m_true=6.0, trial_num=i)

    ps = [params(i) for i in range(ntr)]
    workers.run_efficiency_trials(ps[:64])  # warm-up (library, tables, code objects)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m = workers.run_efficiency_trials(ps)
    e2e = ntr / (time.perf_counter() - t0)

    t0 = time.perf_counter()
    mh = workers.run_efficiency_trials(ps[:nhost], synth="host")
    e2e_host = nhost / (time.perf_counter() - t0)
    dm_host = float(np.max(np.abs(mh - m[:nhost])))

    # device-resident phases: synthesis kernel, then the fit, HIP events on one stream
    cfgs = [dfm.DFMIObject("main_trial", p["laser_config"], p["ifo_config"]) for p in ps]
    x = P.synthesize_asd_trials(cfgs, list(range(ntr)), 0.02)
    g = np.tile([1.6, 6.0, 0.0, 0.0], (ntr, 1))
    F.nls_records(x, 200000.0, 1000.0, 4000, 1, 10, g, parallel=False)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    reps = 3
    ev[0].record(st)
    for _ in range(reps):
        x = P.synthesize_asd_trials(cfgs, list(range(ntr)), 0.02)
    ev[1].record(st)
    for _ in range(reps):
        cols, ok = F.nls_records(x, 200000.0, 1000.0, 4000, 1, 10, g, parallel=False)
    ev[2].record(st)
    torch.cuda.synchronize()
    synth_ms = ev[0].elapsed_time(ev[1]) / reps
    fit_ms = ev[1].elapsed_time(ev[2]) / reps
    assert np.array_equal(cols[1].cpu().numpy(), m)

    # CPU baseline: the reference's per-trial Configure-Simulate-Fit loop, restated
    nb = 200
    t0 = time.perf_counter()
    mc = []
    for p in ps[:nb]:
        cfg = dfm.DFMIObject("main_trial", p["laser_config"], p["ifo_config"])
        xx = np.asarray(P.SignalGenerator().generate(cfg, 0.02, mode="asd", trial_num=p["trial_num"])["main"].samples())
        r = O.fit_chunk((xx.reshape(1, 4000), np.array([1.6, 6.0, 0.0, 0.0]), 10, 1000.0, 200000.0, dict(O.C0)))
        mc.append(r[0][1])
    cpu = nb / (time.perf_counter() - t0)
    dmax = float(np.max(np.abs(np.array(mc) - m[:nb])))
    print(json.dumps({"metric": "efficiency trials/s (one R=4000 buffer each)", "trials": ntr,
                      "end_to_end_trials_per_s": e2e, "end_to_end_host_synth_trials_per_s": e2e_host,
                      "host_synth_sample": nhost, "max_abs_dm_device_vs_host_synth": dm_host,
                      "synth_call_ms": synth_ms, "synth_call_trials_per_s": ntr / (synth_ms / 1e3),
                      "fit_ms": fit_ms, "gpu_fit_only_trials_per_s": ntr / (fit_ms / 1e3),
                      "cpu_baseline": {"value": cpu, "unit": "trials/s", "cores": 1, "kind": "port",
                                       "sample": f"{nb} trials: host simulation + oracle single-buffer fit"},
                      "max_abs_dm_vs_oracle": dmax}), flush=True)


if __name__ == "__main__":
    main()
