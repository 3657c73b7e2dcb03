"""Per-wave finish times of the demodulation kernel (config 2) from the probe buffer:
the spread between the first and the last wave to finish, by XCD. Diagnostic for the
static segment assignment (each wave owns segments s0 + k * waves)."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from deepfmkit_amd import _lib  # noqa: E402
from deepfmkit_amd.fitters import w0_of  # noqa: E402

KW = 16384
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
torch.cuda.synchronize()
_lib.check(lib.dfmi_set_tuning(b"probe", 0), "p")
_lib.check(lib.dfmi_set_tuning(b"probe", 1), "p")
demod()
torch.cuda.synchronize()
n = 16 + 2 * KW
pr = (ctypes.c_int64 * n)()
_lib.check(lib.dfmi_probe_read(pr, n), "read")
_lib.check(lib.dfmi_set_tuning(b"probe", 0), "p")
a = np.frombuffer(pr, dtype=np.int64)
t0 = a[3]
ex = a[16:16 + KW]
xcc = a[16 + KW:16 + 2 * KW]
m = ex > 0
fin = (ex[m] - t0) / 100.0  # us
xc = xcc[m]
nw = int(m.sum())
ws = np.arange(KW)[m]
nsegs = np.array([len(range(w, nseg, nw)) for w in ws])
out = {"waves": nw, "finish_us": {"min": float(fin.min()), "p10": float(np.percentile(fin, 10)),
                                  "median": float(np.median(fin)), "p90": float(np.percentile(fin, 90)),
                                  "max": float(fin.max())},
       "by_xcc_median_us": {int(k): float(np.median(fin[xc == k])) for k in np.unique(xc)},
       "by_xcc_max_us": {int(k): float(fin[xc == k].max()) for k in np.unique(xc)},
       "us_per_segment_median": float(np.median(fin / nsegs)),
       "us_per_segment_p90": float(np.percentile(fin / nsegs, 90))}
print(json.dumps(out), flush=True)
