"""A/B of EKF kernel variants (dfmi_set_tuning keys given as SETTINGS="k=v,k=v;k=v", or
library builds given as LIBS="name=path;name=path", each loaded with its own handle),
interleaved in one process: config 5 (2 s = 400,000 samples @200 kS/s, m=6, 40 dB) for
1 and 64 channels, samples/s per channel, and each variant's max |d state| against the
oracle's scalar C restatement (oracle/csrc/ekf_scalar.c). One JSON line."""
import ctypes
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
    from deepfmkit_amd import _lib
    lib = _lib.load()
    settings = [s for s in os.environ.get("SETTINGS", "ekf_row=1;ekf_row=0").split(";")]
    libs = {}
    if os.environ.get("LIBS"):
        for item in os.environ["LIBS"].split(";"):
            name, path = item.split("=")
            lb = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
            lb.dfmi_ekf_fit.argtypes = lib.dfmi_ekf_fit.argtypes
            lb.dfmi_last_demod_kernel.restype = ctypes.c_char_p
            lb.dfmi_last_error.restype = ctypes.c_char_p
            libs[name] = lb
        settings = list(libs)
    f_samp, f_mod, R = 200000.0, 1000.0, 4000
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("e", laser, ifo, f_samp=f_samp))
    dff.simulate("e", n_seconds=2.0, mode="snr", snr_db=40.0, trial_num=7)
    x1 = np.ascontiguousarray(dff.raws["e"].samples(), dtype=np.float64)
    ns, nb = x1.size, x1.size // R
    cl = ctypes.CDLL(os.path.join(ROOT, "oracle", "libekf_scalar.so"))
    P = ctypes.c_void_p
    cl.ekf_scalar.argtypes = [P, ctypes.c_int64, P, P, P, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                              ctypes.c_int64, ctypes.c_int64, P]
    x0 = np.array([1.6, 6.0, 0.0, 0.0, np.mean(x1)])
    p0, qd = np.ones(5), np.array([1e-8, 1e-8, 1e-6, 1e-6, 1e-8])
    ref = np.zeros((nb, 5))
    cl.ekf_scalar(x1.ctypes.data, ns, x0.ctypes.data, p0.ctypes.data, qd.ctypes.data, float(np.var(x1)),
                  2 * np.pi * f_mod, f_samp, R, nb, ref.ctypes.data)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream()
    init4 = torch.tensor([1.6, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    p0d, qdd = torch.from_numpy(p0).to(dev), torch.from_numpy(qd).to(dev)
    res = {s: {"t1": [], "t64": []} for s in settings}
    xs = {1: torch.from_numpy(x1).to(dev), 64: torch.from_numpy(np.tile(x1, 64)).to(dev)}
    outs = {c: torch.empty((c, nb, 5), dtype=torch.float64, device=dev) for c in (1, 64)}

    cur = {"lib": lib}

    def run(c):
        lb = cur["lib"]
        rc = lb.dfmi_ekf_fit(xs[c].data_ptr(), c, ns, ns, init4.data_ptr(), p0d.data_ptr(), qdd.data_ptr(),
                                    None, 2 * np.pi * f_mod, f_samp, R, nb, outs[c].data_ptr(), 1, st.cuda_stream)
        if rc != 0:
            raise RuntimeError(lb.dfmi_last_error().decode())

    for rnd in range(4):
        for s in settings:
            if libs:
                cur["lib"] = libs[s]
            else:
                for kv in s.split(","):
                    k, v = kv.split("=")
                    _lib.check(lib.dfmi_set_tuning(k.encode(), int(v)), "tune")
            for c in (1, 64):
                run(c)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                run(c)
                torch.cuda.synchronize()
                res[s][f"t{c}"].append(time.perf_counter() - t0)
            res[s]["kernel"] = cur["lib"].dfmi_last_demod_kernel().decode()
            res[s]["max_dstate_vs_c"] = float(np.abs(outs[1][0].cpu().numpy() - ref).max())
            res[s]["max_dstate_64_vs_1"] = float(np.abs(outs[64].cpu().numpy() - outs[1].cpu().numpy()).max())
            res[s]["states1"] = outs[1].cpu().numpy().copy()
    out = {}
    first = res[settings[0]]["states1"]
    for s, r in res.items():
        t1, t64 = float(np.median(r["t1"])), float(np.median(r["t64"]))
        out[s] = {"kernel": r["kernel"], "samples_per_s_1ch": round(ns / t1), "samples_per_s_per_ch_64": round(ns / t64),
                  "max_dstate_vs_c": r["max_dstate_vs_c"], "max_dstate_64_vs_1": r["max_dstate_64_vs_1"],
                  "bit_identical_to_first": bool(np.array_equal(r["states1"], first))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
