"""PCIe-inclusive rate of the headline path: config 2 (100k segments x R = 4000)
handed over as HOST buffers (DFMI_MEM_HOST: the library copies the record to the
device, fits it, copies the 6 result columns + status back and synchronises), from
pinned and from pageable memory. This is the rate a caller with host-resident data
sees; bench.py's `value` is always the HBM-resident one.

One JSON line: segments/s per host-memory kind, the H2D share, and a check that the
results equal the device-resident path's bit for bit."""
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
    from deepfmkit_amd.fitters import w0_of

    lib = _lib.load()
    dev = torch.device("cuda", 0)
    nseg, R, nd = 100_000, 4000, 10
    x_dev = bench.gen_shard(torch, dev, 0, nseg, R, seed=1234)
    w0 = w0_of(1000.0, 200000.0)
    cfg = F.lm_config()
    g = np.array([[1.6, 6.0, 0.0, 0.0]])
    st = torch.cuda.current_stream()
    out_d = torch.empty((6, nseg), dtype=torch.float64, device=dev)
    ok_d = torch.empty(nseg, dtype=torch.int32, device=dev)
    _lib.check(lib.dfmi_nls_record(x_dev.data_ptr(), 1, nseg * R, nseg, R, nd, w0, 0, _lib.ptr(g), 1, nseg - 1, cfg,
                                   out_d.data_ptr(), ok_d.data_ptr(), _lib.DFMI_MEM_DEVICE, st.cuda_stream),
               "dfmi_nls_record")
    torch.cuda.synchronize()
    ref = out_d.cpu().numpy()
    res = {"metric": "segments/s with host-resident input (PCIe-inclusive)", "segments": nseg, "R": R,
           "bytes_h2d": nseg * R * 8}
    for kind in ("pinned", "pageable"):
        xh = x_dev.cpu()
        if kind == "pinned":
            xh = xh.pin_memory()
        out = np.empty((6, nseg))
        ok = np.empty(nseg, dtype=np.int32)

        def call():
            _lib.check(lib.dfmi_nls_record(xh.data_ptr(), 1, nseg * R, nseg, R, nd, w0, 0, _lib.ptr(g), 1, nseg - 1,
                                           cfg, _lib.ptr(out), _lib.ptr(ok), _lib.DFMI_MEM_HOST, None),
                       "dfmi_nls_record")

        call()
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            call()
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        res[kind] = {"seconds": t, "segments_per_s": nseg / t, "h2d_GBps_effective": nseg * R * 8 / t / 1e9,
                     "equal_to_device_path": bool(np.array_equal(out, ref))}
        del xh
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
