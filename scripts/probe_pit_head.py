"""Config 5 (one 400,000-sample channel, m = 6, 40 dB) through the EKF parallel in time per
head length (ekf_pit_head: the samples the sequential EKF runs before the first trajectory is
formed) and block size: call time (HIP events, median of REPS), passes, and the largest state
difference from the default's states. One JSON line per setting.
env: HEADS ("256,128,64,32"), BLOCKS ("0": the default rule), REPS (20), TUNE ("k=v,...": other
tuning keys for the whole run)."""
import ctypes
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
    ns, R = 400_000, 4000
    nb5 = ns // R
    x = torch.empty(ns, dtype=torch.float64, device=dev)
    synth_snr(SnrSpec(seed=bench.SEED, stream=300, f_samp=200000.0, f_mod=1000.0, m=6.0, snr_db=40.0), 0, ns, out=x)
    init4 = torch.tensor([1.6, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    p0d = torch.ones(5, dtype=torch.float64, device=dev)
    qdd = torch.tensor([1e-8, 1e-8, 1e-6, 1e-6, 1e-8], dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = int(os.environ.get("REPS", 20))
    for kv in filter(None, os.environ.get("TUNE", "").split(",")):  # e.g. ekf_pit_topfix=0
        k, v = kv.split("=")
        _lib.check(lib.dfmi_set_tuning(k.encode(), int(v)), k)

    def run(head, block):
        out = torch.empty((1, nb5, 5), dtype=torch.float64, device=dev)
        _lib.check(lib.dfmi_set_tuning(b"ekf_pit_head", head), "head")
        _lib.check(lib.dfmi_set_tuning(b"ekf_pit_block", block), "block")
        try:
            def f():
                _lib.check(lib.dfmi_ekf_fit(x.data_ptr(), 1, ns, ns, init4.data_ptr(), p0d.data_ptr(), qdd.data_ptr(),
                                            None, 2 * np.pi * 1000.0, 200000.0, R, nb5, out.data_ptr(),
                                            _lib.DFMI_MEM_DEVICE, st.cuda_stream), "ekf")
            for _ in range(3):
                f()
            ts = []
            for _ in range(reps):
                ev0.record(st)
                f()
                ev1.record(st)
                ev1.synchronize()
                ts.append(ev0.elapsed_time(ev1))
            passes = (ctypes.c_int32 * 1)()
            _lib.check(lib.dfmi_ekf_pit_passes(ctypes.cast(passes, ctypes.c_void_p), 1), "passes")
            return float(np.median(ts)), int(passes[0]), lib.dfmi_last_demod_kernel().decode(), out
        finally:
            _lib.check(lib.dfmi_set_tuning(b"ekf_pit_head", 256), "head")
            _lib.check(lib.dfmi_set_tuning(b"ekf_pit_block", 0), "block")

    _, _, _, ref = run(256, 0)
    for block in [int(v) for v in os.environ.get("BLOCKS", "0").split(",")]:
        for head in [int(v) for v in os.environ.get("HEADS", "256,128,64,32").split(",")]:
            ms, passes, kn, out = run(head, block)
            print(json.dumps({"head": head, "block": block, "tune": os.environ.get("TUNE", ""), "ms": round(ms, 4),
                              "passes": passes, "kernel": kn,
                              "max_abs_dstate_vs_default": float((out - ref).abs().max().item())}), flush=True)


if __name__ == "__main__":
    main()
