"""Why a config-2 facade call measured 19 ms in one loop and 1.9 ms in another (r04b /
r04c): the same engine call timed in several loop shapes, medians of 7 (ms). One JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import deepfmkit_amd as dfm
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import nls_records, w0_of
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    R, nseg = 4000, 100_000
    x = bench.gen_shard(torch, dev, 0, nseg, R, seed=bench.SEED)
    raw = dfm.DeepRawObject(x)
    raw.f_samp, raw.f_mod, raw.label = 200000.0, 1000.0, "c2"
    dff = dfm.DeepFitFramework()
    dff.raws["c2"] = raw
    out = torch.empty((6, nseg), dtype=torch.float64, device=dev)
    ok = torch.empty(nseg, dtype=torch.int32, device=dev)
    g = np.array([1.6, 6.0, 0.0, 0.0])
    st = torch.cuda.current_stream()
    cfg = F.lm_config()

    def raw_call():
        _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nseg * R, nseg, R, 10, w0_of(1000.0, 200000.0), 0, _lib.ptr(g),
                                       1, nseg - 1, cfg, out.data_ptr(), ok.data_ptr(), _lib.DFMI_MEM_DEVICE,
                                       st.cuda_stream), "nls")

    def timed(fn, pre=None, post=None, n=7):
        ts = []
        for _ in range(n):
            if pre:
                pre()
            t0 = time.perf_counter()
            fn()
            if post:
                post()
            ts.append(time.perf_counter() - t0)
        return round(float(np.median(ts)) * 1e3, 3)

    sync = torch.cuda.synchronize
    for _ in range(3):
        raw_call()
    sync()
    res = {
        "raw_call+sync": timed(raw_call, post=sync),
        "raw_call+sync, sync before": timed(raw_call, pre=sync, post=sync),
        "nls_records+sync": timed(lambda: nls_records(x.reshape(1, -1), 200000.0, 1000.0, R, nseg), post=sync),
        "nls_records+cpu()": timed(lambda: [t.cpu() for t in nls_records(x.reshape(1, -1), 200000.0, 1000.0, R, nseg)]),
        "facade": timed(lambda: dff.fit("c2", n=20, fit_label="e")),
        "facade, sync before": timed(lambda: dff.fit("c2", n=20, fit_label="e"), pre=sync),
        "raw_call+sync again": timed(raw_call, post=sync),
        "sleep 1ms then raw_call+sync": timed(raw_call, pre=lambda: time.sleep(1e-3), post=sync),
        "sleep 20ms then raw_call+sync": timed(raw_call, pre=lambda: time.sleep(2e-2), post=sync),
    }
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    sync()
    e0.record(st)
    raw_call()
    e1.record(st)
    sync()
    res["events_one_call"] = round(e0.elapsed_time(e1), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
