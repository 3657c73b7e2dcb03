"""Wall time of one config-2 dfmi_nls_record (100,000 x R=4000, device-resident record) per
output mode: DFMI_MEM_DEVICE (+ a torch D2H of the results into pinned memory),
DFMI_MEM_DEVICE | DFMI_MEM_OUT_HOST with and without the split copy (tuning key out_split).
One JSON line per mode (median of 11 calls after 3 warm ones)."""
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
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    lib = _lib.load()
    R, nbuf = 4000, int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    x = bench.gen_shard(torch, torch.device("cuda", 0), 0, nbuf, R, seed=bench.SEED)
    g = np.array([1.6, 6.0, 0.0, 0.0])
    w0 = 2.0 * np.pi * 1000.0 / 200000.0
    st = torch.cuda.current_stream()
    od = torch.empty((7, nbuf), dtype=torch.float64, device="cuda")
    kd = torch.empty(nbuf, dtype=torch.int32, device="cuda")
    oh = torch.empty((7, nbuf), dtype=torch.float64, pin_memory=True)
    kh = torch.empty(nbuf, dtype=torch.int32, pin_memory=True)

    def dev_mode():
        _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nbuf * R, nbuf, R, 10, w0, 0, _lib.ptr(g), 1, nbuf - 1,
                                       F.lm_config(), od.data_ptr(), kd.data_ptr(), _lib.DFMI_MEM_DEVICE,
                                       st.cuda_stream), "d")
        od[6].view(torch.int64).copy_(kd)
        oh.copy_(od, non_blocking=True)
        st.synchronize()

    def host_mode():
        _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nbuf * R, nbuf, R, 10, w0, 0, _lib.ptr(g), 1, nbuf - 1,
                                       F.lm_config(), oh.data_ptr(), kh.data_ptr(),
                                       _lib.DFMI_MEM_DEVICE | _lib.DFMI_MEM_OUT_HOST, st.cuda_stream), "h")
        st.synchronize()

    def kernels_only():
        _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nbuf * R, nbuf, R, 10, w0, 0, _lib.ptr(g), 1, nbuf - 1,
                                       F.lm_config(), od.data_ptr(), kd.data_ptr(), _lib.DFMI_MEM_DEVICE,
                                       st.cuda_stream), "d")
        st.synchronize()

    def run(name, fn, **tune):
        for k, v in tune.items():
            _lib.check(lib.dfmi_set_tuning(k.encode(), v), "tune")
        for _ in range(3):
            fn()
        ts = []
        for _ in range(11):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        kn = lib.dfmi_last_demod_kernel().decode()
        print(json.dumps({"mode": name, "ms": round(float(np.median(ts)) * 1e3, 4), "min_ms": round(min(ts) * 1e3, 4),
                          "kernel": kn, **tune}), flush=True)
        for k in tune:
            _lib.check(lib.dfmi_set_tuning(k.encode(), 1), "tune")

    only = sys.argv[2] if len(sys.argv) > 2 else ""
    if only in ("", "kernels"):
        run("kernels_only (DFMI_MEM_DEVICE, sync)", kernels_only)
    if only in ("", "device"):
        run("DFMI_MEM_DEVICE + torch D2H", dev_mode)
    if only in ("", "split"):
        run("DFMI_MEM_DEVICE|OUT_HOST split", host_mode, out_split=1)
    if only in ("", "nosplit"):
        run("DFMI_MEM_DEVICE|OUT_HOST no split", host_mode, out_split=0)


if __name__ == "__main__":
    main()
