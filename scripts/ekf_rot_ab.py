"""A/B of the EKF kernels inside one process (config 5: 2 s = 400,000 samples, m = 6, 40 dB,
R = 4000; KERNELS="rot,row" by default, also lanerot, lane): ekf_rot_kernel (sincos by
rotation between anchors, tuning ekf_rot 1) vs ekf_row_kernel (full sincos per sample,
ekf_rot 0), or the lane kernels likewise (ekf_row 0), interleaved, median of `reps` per
setting and channel count; states of every variant against the scalar C restatement of
EKFFitter.fit (oracle/csrc/ekf_scalar.c) for channel 0. One JSON line per channel count.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--channels", default="1,4,64,1024")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--f-samp", type=float, default=200000.0)
    ap.add_argument("--f-mod", type=float, default=1000.0)
    ap.add_argument("--m", type=float, default=6.0)
    ap.add_argument("--seconds", type=float, default=2.0)
    args = ap.parse_args()
    import torch

    from deepfmkit_amd import _lib
    from deepfmkit_amd.physics import SnrSpec, synth_snr

    lib = _lib.load()
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    fs, fm = args.f_samp, args.f_mod
    R = int(round(fs / fm * 20))
    ns = int(args.seconds * fs)
    nb = ns // R
    p0, qd = np.ones(5), np.array([1e-8, 1e-8, 1e-6, 1e-6, 1e-8])
    init4 = torch.tensor([1.6, args.m, 0.0, 0.0], dtype=torch.float64, device=dev)
    p0d, qdd = torch.from_numpy(p0).to(dev), torch.from_numpy(qd).to(dev)
    cl = ctypes.CDLL(os.path.join(ROOT, "oracle", "libekf_scalar.so"))
    P_ = ctypes.c_void_p
    cl.ekf_scalar.argtypes = [P_, ctypes.c_int64, P_, P_, P_, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                              ctypes.c_int64, ctypes.c_int64, P_]
    allk = {"rot": (1, 1), "row": (1, 0), "lanerot": (0, 1), "lane": (0, 0)}
    settings = {k: allk[k] for k in os.environ.get("KERNELS", "rot,row").split(",")}
    for nch in [int(c) for c in args.channels.split(",")]:
        xe = torch.empty(nch * ns, dtype=torch.float64, device=dev)
        for c in range(nch):
            synth_snr(SnrSpec(seed=1234, stream=100 + c, f_samp=fs, f_mod=fm, m=args.m, snr_db=40.0), 0, ns,
                      out=xe[c * ns:(c + 1) * ns])
        stt = torch.empty((nch, nb, 5), dtype=torch.float64, device=dev)
        x1 = xe[:ns].cpu().numpy()
        cst = np.zeros((nb, 5))
        cl.ekf_scalar(x1.ctypes.data, ns, np.array([1.6, args.m, 0.0, 0.0, np.mean(x1)]).ctypes.data,
                      p0.ctypes.data, qd.ctypes.data, float(np.var(x1)), 2 * np.pi * fm, fs, R, nb, cst.ctypes.data)
        times = {k: [] for k in settings}
        res = {}
        for rep in range(args.reps + 1):
            for name, (row, rot) in settings.items():
                _lib.check(lib.dfmi_set_tuning(b"ekf_row", row), "tune")
                _lib.check(lib.dfmi_set_tuning(b"ekf_rot", rot), "tune")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record(stream)
                _lib.check(lib.dfmi_ekf_fit(xe.data_ptr(), nch, ns, ns, init4.data_ptr(), p0d.data_ptr(),
                                            qdd.data_ptr(), None, 2 * np.pi * fm, fs, R, nb, stt.data_ptr(),
                                            _lib.DFMI_MEM_DEVICE, stream.cuda_stream), "dfmi_ekf_fit")
                e1.record(stream)
                torch.cuda.synchronize()
                if rep:
                    times[name].append(e0.elapsed_time(e1) * 1e-3)
                s = stt.cpu().numpy()
                res[name] = (lib.dfmi_last_demod_kernel().decode(), float(np.max(np.abs(s[0] - cst))), s)
        _lib.check(lib.dfmi_set_tuning(b"ekf_row", 1), "tune")
        _lib.check(lib.dfmi_set_tuning(b"ekf_rot", 1), "tune")
        line = {"channels": nch, "n_samp": ns, "f_samp": fs, "f_mod": fm, "m": args.m}
        for name in settings:
            t = float(np.median(times[name]))
            line[name] = {"kernel": res[name][0], "s": round(t, 6), "samples_per_s_per_channel": round(ns / t, 1),
                          "max_abs_dstate_ch0_vs_c": res[name][1]}
        names = list(settings)
        line[f"max_abs_{names[0]}_vs_{names[-1]}_all_channels"] = float(np.max(np.abs(res[names[0]][2] -
                                                                                   res[names[-1]][2])))
        print(json.dumps(line), flush=True)
        del xe, stt


if __name__ == "__main__":
    main()
