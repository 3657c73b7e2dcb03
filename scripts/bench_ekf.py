"""Config 5 (BASELINE.json): the EKF time-domain path (EKFFitter, fitters.py:214-320,
notebooks/2.0_EKF) on the GPU — one lane per channel, a serial predict/update
chain over the samples — next to the CPU oracle (oracle/nls_oracle.py ekf_record,
the restated reference loop, one core).

Workload: `channels` independent snr-mode records (f_samp 200 kHz, f_mod 1 kHz,
m = 6, 40 dB, n = 20 -> R = 4000 snapshot spacing) of `seconds` each, resident in
HBM. Timing: HIP events around one dfmi_ekf_fit call (median of `reps`), which
includes the per-record pre-reductions (np.mean, np.var: fitters.py:253, 256) on the
device. Reported: samples/s per channel (the serial chain's speed) and aggregate
samples/s. One JSON line per channel count.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--channels", default="1,64,1024", help="comma- or colon-separated channel counts")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=0.1, help="oracle sample length (s of signal)")
    args = ap.parse_args()
    import torch

    import deepfmkit_amd as dfm
    from deepfmkit_amd import _lib
    from oracle import nls_oracle as O

    f_samp, f_mod, n = 200000.0, 1000.0, 20
    R = int(f_samp / f_mod * n)
    laser = dfm.LaserConfig()
    ifo = dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("ekf", laser, ifo, f_samp=f_samp))
    dff.simulate("ekf", n_seconds=args.seconds, mode="snr", snr_db=40.0, trial_num=0)
    x1 = np.asarray(dff.raws["ekf"].samples(), dtype=np.float64)
    ns = x1.size
    nbuf = ns // R

    ncpu = int(args.cpu_seconds * f_samp)
    t0 = time.perf_counter()
    ref = O.ekf_record(x1[:ncpu], f_samp, f_mod, n)
    cpu_rate = ncpu / (time.perf_counter() - t0)
    cpu = {"value": cpu_rate, "unit": "samples/s per channel", "cores": 1, "kind": "port",
           "sample": f"{ncpu} samples ({args.cpu_seconds} s of signal), oracle restatement of EKFFitter.fit"}

    # second CPU baseline: the scalar C restatement of the same loop
    # (oracle/csrc/ekf_scalar.c, libm sin / cos, one core) over the whole record
    import ctypes
    cl = ctypes.CDLL(os.path.join(ROOT, "oracle", "libekf_scalar.so"))
    P_ = ctypes.c_void_p
    cl.ekf_scalar.argtypes = [P_, ctypes.c_int64, P_, P_, P_, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                              ctypes.c_int64, ctypes.c_int64, P_]
    cx0 = np.array([1.6, 6.0, 0.0, 0.0, np.mean(x1)])
    cp0, cq = np.ones(5), np.array([1e-8, 1e-8, 1e-6, 1e-6, 1e-8])
    cst = np.zeros((nbuf, 5))
    t0 = time.perf_counter()
    cl.ekf_scalar(x1.ctypes.data, ns, cx0.ctypes.data, cp0.ctypes.data, cq.ctypes.data, float(np.var(x1)),
                  2 * np.pi * f_mod, f_samp, R, nbuf, cst.ctypes.data)
    c_rate = ns / (time.perf_counter() - t0)
    refc = O.ekf_record(x1[:ncpu], f_samp, f_mod, n)
    cpart = np.zeros((ncpu // R, 5))
    cx0p = np.array([1.6, 6.0, 0.0, 0.0, np.mean(x1[:ncpu])])
    cl.ekf_scalar(x1.ctypes.data, ncpu, cx0p.ctypes.data, cp0.ctypes.data, cq.ctypes.data, float(np.var(x1[:ncpu])),
                  2 * np.pi * f_mod, f_samp, R, ncpu // R, cpart.ctypes.data)
    cpu_c = {"value": c_rate, "unit": "samples/s per channel", "cores": 1, "kind": "port",
             "sample": f"{ns} samples, oracle/csrc/ekf_scalar.c (gcc -O2, libm), the numpy loop's operation order",
             "max_abs_dstate_vs_oracle": float(np.max(np.abs(cpart - refc)))}

    lib = _lib.load()
    dev = torch.device("cuda:0")
    # parity on the oracle's own record (the prefix, with ITS mean and variance as x0[4]
    # and R: fitters.py:253, 256), through the drop-in facade
    raw = dfm.DeepRawObject(data=x1[:ncpu])
    raw.f_samp, raw.f_mod = f_samp, f_mod
    got = dfm.fitters.ekf_records([raw], n)[0]
    parity = float(np.max(np.abs(got - ref)))
    st = torch.cuda.current_stream()
    p0 = torch.ones(5, dtype=torch.float64, device=dev)
    qd = torch.tensor([1e-8, 1e-8, 1e-6, 1e-6, 1e-8], dtype=torch.float64, device=dev)
    init4 = torch.tensor([1.6, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    for nch in [int(v) for v in args.channels.replace(":", ",").split(",")]:
        x = torch.from_numpy(x1).to(dev).reshape(1, -1).expand(nch, -1).contiguous()
        states = torch.empty((nch, nbuf, 5), dtype=torch.float64, device=dev)

        def call():
            # EKFFitter.fit whole: np.mean / np.var of every channel on the device, then the chain
            _lib.check(lib.dfmi_ekf_fit(x.data_ptr(), nch, ns, ns, init4.data_ptr(), p0.data_ptr(), qd.data_ptr(),
                                        None, 2 * np.pi * f_mod, f_samp, R, nbuf, states.data_ptr(),
                                        _lib.DFMI_MEM_DEVICE, st.cuda_stream), "dfmi_ekf_fit")

        call()
        torch.cuda.synchronize()
        times = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            call()
            e1.record(st)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / 1e3)
        t = float(np.median(times))
        print(json.dumps({"metric": "EKF samples/s", "channels": nch, "samples_per_channel": ns, "seconds": t,
                          "per_channel_samples_per_s": ns / t, "aggregate_samples_per_s": nch * ns / t,
                          "max_abs_dstate_vs_oracle": parity, "parity_record": f"{ncpu} samples", "cpu_baseline": cpu,
                          "cpu_baseline_c_scalar": cpu_c,
                          "data": "snr-mode m=6, 40 dB, 200 kS/s (the package's bit-exact physics.py restatement)"}),
              flush=True)
        del x


if __name__ == "__main__":
    main()
