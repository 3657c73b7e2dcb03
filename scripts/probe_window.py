"""Per-window step time in ONE process (config 2): is the driver's 20-step window
slower than 100 steps because of a one-time cost (first launches after a sync,
clock ramp) or steady-state noise? Prints ms/step for successive windows."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from deepfmkit_amd import _lib  # noqa: E402
from deepfmkit_amd import fit as F  # noqa: E402
from deepfmkit_amd.fitters import w0_of  # noqa: E402

lib = _lib.load()
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
R, nd, nseg = 4000, 10, 100_000
x = bench.gen_shard(torch, dev, 0, nseg, R, seed=bench.SEED)
cfg = F.lm_config()
g = np.ascontiguousarray([[1.6, 6.0, 0.0, 0.0]])
out = torch.empty((6, nseg), dtype=torch.float64, device=dev)
ok = torch.empty(nseg, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream()
w0 = w0_of(1000.0, 200000.0)


def step():
    _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nseg * R, nseg, R, nd, w0, 0, _lib.ptr(g), 1, nseg - 1, cfg,
                                   out.data_ptr(), ok.data_ptr(), 1, st.cuda_stream), "nls")


def window(k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


res = {"first_call_ms": window(1)}
res["warm5"] = window(5)
for i, k in enumerate([20, 20, 100, 20, 5, 1, 20]):
    res[f"w{i}_{k}"] = round(window(k), 4)
# host launch cost per call (no sync): enqueue time of 20 calls
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    step()
res["host_enqueue_ms_per_call"] = round((time.perf_counter() - t0) / 20 * 1e3, 4)
torch.cuda.synchronize()
# events around 20 steps (device time only)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for _ in range(20):
    step()
e1.record(st)
e1.synchronize()
res["events_ms_per_step_20"] = round(e0.elapsed_time(e1) / 20, 4)
print(json.dumps(res))
