"""Config 5, one channel: the EKF parallel in time (ekf_pit.h) at several block sizes against
the sequential row kernel (ekf_rot_kernel). Input resident in HBM (dfmi_ekf_fit, device
memory, the bench's call); HIP-event time per call (median of REPS), the passes each
variant ran and its largest state difference from the sequential kernel. One JSON line.

FUSED: ekf_pit_fused (default 1). PASSES: ekf_pit_passes (default 12). PITMIN: ekf_pit_min for the parallel variants. SECONDS_: record length. VARIANTS: comma list of block:head pairs (ekf_pit_block, 0 = auto; ekf_pit_head samples).
CHANNELS: channel counts.
"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from deepfmkit_amd import _lib
    from deepfmkit_amd.physics import SnrSpec, synth_snr
    lib = _lib.load()
    dev = torch.device("cuda:0")
    F_SAMP, F_MOD, R = 200000.0, 1000.0, int(os.environ.get("R_", "4000"))
    ns = int(float(os.environ.get("SECONDS_", "2.0")) * F_SAMP)
    nb5 = ns // R
    reps = int(os.environ.get("REPS", "5"))
    variants = [tuple(int(v) for v in p.split(":")) for p in os.environ.get("VARIANTS", "0:512,0:0,25:512,49:1024").split(",")]
    chans = [int(c) for c in os.environ.get("CHANNELS", "1").split(",")]
    init4 = torch.tensor([1.6, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    p0 = torch.ones(5, dtype=torch.float64, device=dev)
    qd = torch.tensor([1e-8, 1e-8, 1e-6, 1e-6, 1e-8], dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream()
    out = {"workload": f"EKFFitter.fit, {ns} samples @200 kS/s, m=6, 40 dB, R={R}", "variants": []}
    for nch in chans:
        xe = torch.empty(nch * ns, dtype=torch.float64, device=dev)
        for c in range(nch):
            synth_snr(SnrSpec(seed=1234, stream=100 + c, f_samp=F_SAMP, f_mod=F_MOD, m=6.0, snr_db=40.0), 0, ns,
                      out=xe[c * ns:(c + 1) * ns])
        stt = torch.empty((nch, nb5, 5), dtype=torch.float64, device=dev)

        def call():
            _lib.check(lib.dfmi_ekf_fit(xe.data_ptr(), nch, ns, ns, init4.data_ptr(), p0.data_ptr(), qd.data_ptr(),
                                        None, 2 * np.pi * F_MOD, F_SAMP, R, nb5, stt.data_ptr(), _lib.DFMI_MEM_DEVICE,
                                        stream.cuda_stream), "dfmi_ekf_fit")

        def timed():
            call()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                call()
                b.record(stream)
                b.synchronize()
                ts.append(a.elapsed_time(b))
            return float(np.median(ts))

        _lib.check(lib.dfmi_set_tuning(b"ekf_pit", 0), "tune")
        tseq = timed()
        seq = stt.cpu().numpy().copy()
        out["variants"].append({"channels": nch, "kernel": lib.dfmi_last_demod_kernel().decode(), "ms": round(tseq, 4),
                                "samples_per_s_per_channel": round(ns / tseq * 1e3, 1)})
        _lib.check(lib.dfmi_set_tuning(b"ekf_pit", 1024), "tune")
        _lib.check(lib.dfmi_set_tuning(b"ekf_pit_min", int(os.environ.get("PITMIN", "32768"))), "tune")
        _lib.check(lib.dfmi_set_tuning(b"ekf_pit_fused", int(os.environ.get("FUSED", "1"))), "tune")
        _lib.check(lib.dfmi_set_tuning(b"ekf_pit_passes", int(os.environ.get("PASSES", "12"))), "tune")
        for B, head in variants:
            _lib.check(lib.dfmi_set_tuning(b"ekf_pit_block", B), "tune")
            _lib.check(lib.dfmi_set_tuning(b"ekf_pit_head", head), "tune")
            t = timed()
            passes = (ctypes.c_int32 * nch)()
            _lib.check(lib.dfmi_ekf_pit_passes(ctypes.cast(passes, ctypes.c_void_p), nch), "passes")
            got = stt.cpu().numpy()
            out["variants"].append({"channels": nch, "head": head, "kernel": lib.dfmi_last_demod_kernel().decode(), "ms": round(t, 4),
                                    "samples_per_s_per_channel": round(ns / t * 1e3, 1),
                                    "passes": sorted(set(passes)), "speedup_vs_seq": round(tseq / t, 2),
                                    "max_abs_dstate_vs_seq": float(np.max(np.abs(got - seq)))})
            print(json.dumps(out["variants"][-1]), flush=True)
        _lib.check(lib.dfmi_set_tuning(b"ekf_pit_block", 0), "tune")
        _lib.check(lib.dfmi_set_tuning(b"ekf_pit_head", 256), "tune")
        _lib.check(lib.dfmi_set_tuning(b"ekf_pit", 1024), "tune")
        _lib.check(lib.dfmi_set_tuning(b"ekf_pit_min", 4096), "tune")
        _lib.check(lib.dfmi_set_tuning(b"ekf_pit_passes", 12), "tune")
        del xe, stt
    print(json.dumps(out))


if __name__ == "__main__":
    main()
