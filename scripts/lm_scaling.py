"""LM kernel time vs batch size (dfmi_lm on QI from dfmi_demod, every segment its own
chunk, guess = the true parameters' neighbourhood): separates a latency-bound kernel
(time flat while waves <= SIMDs) from a throughput-bound one (time ~ segments)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from deepfmkit_amd import _lib  # noqa: E402
from deepfmkit_amd import fit as F  # noqa: E402
from deepfmkit_amd.fitters import w0_of  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
R, nd = 4000, 10
w0 = w0_of(1000.0, 200000.0)
st = torch.cuda.current_stream()
cfg = F.lm_config()
out = {}
for nseg in (1024, 16384, 32768, 65536, 100000, 200000):
    x = bench.gen_shard(torch, dev, 0, nseg, R, seed=1)
    qi = torch.empty((2 * nd, nseg), dtype=torch.float64, device=dev)
    dc = torch.empty(nseg, dtype=torch.float64, device=dev)
    _lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0, 0, qi.data_ptr(), dc.data_ptr(), 1, st.cuda_stream),
               "demod")
    del x
    g = torch.tensor([1.0, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev).repeat(nseg, 1).contiguous()
    p = torch.empty((4, nseg), dtype=torch.float64, device=dev)
    ssq = torch.empty(nseg, dtype=torch.float64, device=dev)
    status = torch.empty(nseg, dtype=torch.int32, device=dev)

    def lm():
        _lib.check(lib.dfmi_lm(qi.data_ptr(), nseg, nd, g.data_ptr(), 1, nseg, cfg, p.data_ptr(), ssq.data_ptr(),
                               status.data_ptr(), 1, st.cuda_stream), "lm")

    lm()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(10):
        lm()
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    out[nseg] = {"ms": round(ms, 4), "waves": (nseg + 63) // 64, "ns_per_segment": round(ms * 1e6 / nseg, 2),
                 "status0": float((status == 0).float().mean().item())}
print(json.dumps(out, indent=1))
