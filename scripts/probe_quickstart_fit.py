"""The reference quickstart's own fit (notebooks/0.0_quickstart.ipynb cell 0: 10 s at 200 kS/s,
m = 31.4, 500 buffers of R = 4000) timed on the GPU: dfmi_nls_record over the device-resident
record (parallel, chunk size 1: the seed, the demodulation and 499 LM fits, a latency-bound
launch), per tuning set, at ndata 62 and 30; and DeepFitFramework.fit end to end (the
notebook's call). One JSON line per measurement.
env: SETS (';'-separated tuning sets 'key=v,key=v'; default: the defaults), REPS (50)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import w0_of
    from test_gpu_quickstart import quickstart_framework
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    dff, label, _ = quickstart_framework()
    x_host = np.ascontiguousarray(dff.raws[label].samples(), dtype=np.float64)
    R, nbuf = 4000, x_host.size // 4000
    x = torch.from_numpy(x_host[:nbuf * R].copy()).to(dev)
    cfg = F.lm_config()
    guess = np.array([1.6, 6.0, 0.0, 0.0])
    out = torch.empty((6, nbuf), dtype=torch.float64, device=dev)
    ok = torch.empty(nbuf, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = int(os.environ.get("REPS", 50))
    sets = [s for s in os.environ.get("SETS", "").split(";")]
    for spec in sets:
        tune = dict(kv.split("=") for kv in filter(None, spec.split(",")))
        olds = {}
        for k, v in tune.items():
            o = ctypes_get(lib, _lib, k)
            olds[k] = o
            _lib.check(lib.dfmi_set_tuning(k.encode(), int(v)), k)
        try:
            for nd in (62, 30):
                def step():
                    _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nbuf * R, nbuf, R, nd, w0_of(1000.0, 200000.0), 0,
                                                   _lib.ptr(guess), 1, nbuf - 1, cfg, out.data_ptr(), ok.data_ptr(),
                                                   _lib.DFMI_MEM_DEVICE, st.cuda_stream), "dfmi_nls_record")
                for _ in range(5):
                    step()
                ev0.record(st)
                for _ in range(reps):
                    step()
                ev1.record(st)
                ev1.synchronize()
                ms = ev0.elapsed_time(ev1) / reps
                print(json.dumps({"what": "dfmi_nls_record", "ndata": nd, "tune": tune, "ms": round(ms, 4),
                                  "kernel": lib.dfmi_last_demod_kernel().decode(),
                                  "status": np.bincount(ok.cpu().numpy(), minlength=3).tolist()}), flush=True)
        finally:
            for k, v in olds.items():
                _lib.check(lib.dfmi_set_tuning(k.encode(), int(v)), k)
    for nd in (62, 30):  # the notebook's own call, host record through the facade
        dff.fit(label, ndata=nd)
        t = []
        for _ in range(5):
            t0 = time.perf_counter()
            dff.fit(label, ndata=nd)
            t.append(time.perf_counter() - t0)
        print(json.dumps({"what": "DeepFitFramework.fit (host record)", "ndata": nd, "ms": round(min(t) * 1e3, 3)}),
              flush=True)


def ctypes_get(lib, _lib, key):
    import ctypes
    v = ctypes.c_int64()
    _lib.check(lib.dfmi_get_tuning(key.encode(), ctypes.byref(v)), key)
    return v.value


if __name__ == "__main__":
    main()
