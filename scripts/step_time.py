"""ms/step of the config-2 record pipeline (dfmi_nls_record, 100k segments) for one build
of libdfmi.so (LIB=<path>; default the in-tree library): 10 warm-up steps, then the
median of 5 windows of 20 steps, plus the demodulation kernel alone (HIP events)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from deepfmkit_amd import _lib  # noqa: E402

if os.environ.get("LIB"):
    _lib.LIB_PATH = os.path.abspath(os.environ["LIB"])
import bench  # noqa: E402
from deepfmkit_amd import fit as F  # noqa: E402
from deepfmkit_amd.fitters import w0_of  # noqa: E402

lib = _lib.load()
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
nseg, R, nd = 100_000, 4000, 10
x = bench.gen_shard(torch, dev, 0, nseg, R, seed=bench.SEED)
st = torch.cuda.current_stream()
w0 = w0_of(1000.0, 200000.0)
cfg = F.lm_config()
g = np.array([1.6, 6.0, 0.0, 0.0])
out = torch.empty((6, nseg), dtype=torch.float64, device=dev)
ok = torch.empty(nseg, dtype=torch.int32, device=dev)
rows = torch.empty((nseg, lib.dfmi_qi_row_stride(nd)), dtype=torch.float64, device=dev)


def step():
    _lib.check(lib.dfmi_nls_record(x.data_ptr(), 1, nseg * R, nseg, R, nd, w0, 0, _lib.ptr(g), 1, nseg - 1, cfg,
                                   out.data_ptr(), ok.data_ptr(), _lib.DFMI_MEM_DEVICE, st.cuda_stream), "rec")


def demod():
    _lib.check(lib.dfmi_demod_rows(x.data_ptr(), nseg, R, R, nd, w0, 0, rows.data_ptr(), _lib.DFMI_MEM_DEVICE,
                                   st.cuda_stream), "demod")


def timed(fn, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(n):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / n


for _ in range(10):
    step()
torch.cuda.synchronize()
steps = [timed(step, 20) for _ in range(5)]
dem = [timed(demod, 20) for _ in range(3)]
res = torch.cat([out.flatten(), ok.double()]).sum().item()
print(json.dumps({"lib": os.path.basename(_lib.LIB_PATH), "ms_per_step": round(float(np.median(steps)), 4),
                  "demod_ms": round(float(np.median(dem)), 4), "checksum": res}), flush=True)
