"""Where the demodulation kernel's time goes (config 2): dfmi_set_tuning("probe", 1)
timestamps (s_memrealtime, 100 MHz) at the entry of workgroup 0 and of the last
workgroup and at the exit of workgroup 0's first wave, against the kernel duration
(HIP events): dispatch spread, one wave's busy time, and the drain."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from deepfmkit_amd import _lib  # noqa: E402
from deepfmkit_amd.fitters import w0_of  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
nseg, R, nd = int(os.environ.get("NSEG", 100000)), 4000, 10
x = bench.gen_shard(torch, dev, 0, nseg, R, seed=bench.SEED)
st = torch.cuda.current_stream()
rows = torch.empty((nseg, lib.dfmi_qi_row_stride(nd)), dtype=torch.float64, device=dev)


def demod():
    _lib.check(lib.dfmi_demod_rows(x.data_ptr(), nseg, R, R, nd, w0_of(1000.0, 200000.0), 0, rows.data_ptr(),
                                   _lib.DFMI_MEM_DEVICE, st.cuda_stream), "demod")


for _ in range(5):
    demod()
out = []
for rep in range(3):
    _lib.check(lib.dfmi_set_tuning(b"probe", 0), "p")
    _lib.check(lib.dfmi_set_tuning(b"probe", 1), "p")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    demod()
    e1.record(st)
    torch.cuda.synchronize()
    pr = (ctypes.c_int64 * 16)()
    _lib.check(lib.dfmi_probe_read(pr, 16), "read")
    ms = e0.elapsed_time(e1)
    out.append({"kernel_ms": round(ms, 4), "dispatch_spread_us": (pr[4] - pr[3]) / 100.0,
                "wg0_wave0_busy_us": (pr[5] - pr[3]) / 100.0})
_lib.check(lib.dfmi_set_tuning(b"probe", 0), "p")
print(json.dumps({"kernel": lib.dfmi_last_demod_kernel().decode(), "segments": nseg, "runs": out}), flush=True)
