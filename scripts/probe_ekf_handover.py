"""The EKF parallel in time's hand-over (round 6), by variant: a batch of NCH config-5 channels
(400,000 samples, m = 6, 40 dB) with NBAD m = 20 channels fitted from init_m = 6 (never lock)
spread among them. Per ekf_pit_overlap (3: re-runs launched at the host check on the next of a
pool of high-priority streams beside the passes; 2: one high-priority stream; 1: one
default-priority stream; 0: after the passes, on the caller's stream) the batch time, against the passes alone (ekf_pit_seq 0) and the NBAD
channels' sequential run alone (ekf_pit 0). One JSON line per measurement.
env: NCH (1024), NBAD (64), NS (400000), MODES ("3,2,0"), REPS (2)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from deepfmkit_amd import _lib
    from deepfmkit_amd.physics import SnrSpec, synth_snr
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    nch, nbad, ns = int(os.environ.get("NCH", 1024)), int(os.environ.get("NBAD", 64)), int(os.environ.get("NS", 400000))
    reps = int(os.environ.get("REPS", 2))
    R = 4000
    nb5 = ns // R
    ms = [6.0] * nch
    for i in range(nbad):
        ms[(i * nch) // max(nbad, 1) + 3] = 20.0
    xe = torch.empty(nch * ns, dtype=torch.float64, device=dev)
    for c, m in enumerate(ms):
        synth_snr(SnrSpec(seed=bench.SEED, stream=300 + c, f_samp=200000.0, f_mod=1000.0, m=m, snr_db=40.0), 0, ns,
                  out=xe[c * ns:(c + 1) * ns])
    init4 = torch.tensor([1.6, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    p0d = torch.ones(5, dtype=torch.float64, device=dev)
    qdd = torch.tensor([1e-8, 1e-8, 1e-6, 1e-6, 1e-8], dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run(x, n, tune):
        out = torch.empty((n, nb5, 5), dtype=torch.float64, device=dev)
        for k, v in tune.items():
            _lib.check(lib.dfmi_set_tuning(k.encode(), v), k)
        try:
            def f():
                _lib.check(lib.dfmi_ekf_fit(x.data_ptr(), n, ns, ns, init4.data_ptr(), p0d.data_ptr(), qdd.data_ptr(),
                                            None, 2 * np.pi * 1000.0, 200000.0, R, nb5, out.data_ptr(),
                                            _lib.DFMI_MEM_DEVICE, st.cuda_stream), "ekf")
            f()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                ev0.record(st)
                f()
                ev1.record(st)
                ev1.synchronize()
                ts.append(ev0.elapsed_time(ev1))
            return min(ts), lib.dfmi_last_demod_kernel().decode(), out
        finally:
            for k in tune:
                _lib.check(lib.dfmi_set_tuning(k.encode(), {"ekf_pit": 1024, "ekf_pit_seq": 1,
                                                            "ekf_pit_overlap": 0}[k]), k)
    res = {}
    for mode in [int(v) for v in os.environ.get("MODES", "3,2,0").split(",")]:
        t, kn, out = run(xe, nch, {"ekf_pit_overlap": mode})
        res[mode] = out
        print(json.dumps({"what": "batch", "overlap": mode, "channels": nch, "non_locking": nbad,
                          "ms": round(t, 3), "kernel": kn}), flush=True)
    t, kn, _ = run(xe, nch, {"ekf_pit_seq": 0})
    print(json.dumps({"what": "passes alone (ekf_pit_seq 0)", "ms": round(t, 3), "kernel": kn}), flush=True)
    idx = [i for i, m in enumerate(ms) if m != 6.0]
    if not idx:
        return
    xs = torch.stack([xe[i * ns:(i + 1) * ns] for i in idx]).reshape(-1).contiguous()
    t, kn, sq = run(xs, len(idx), {"ekf_pit": 0})
    print(json.dumps({"what": "handed-over channels alone, sequential", "ms": round(t, 3), "kernel": kn,
                      "equal_to_batch_states": {m: bool(torch.equal(r[idx], sq)) for m, r in res.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
