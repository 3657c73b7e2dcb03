"""Diagnostics of the refill LM kernel (csrc/lm_refill.h): passes per wave, busy lanes per
pass, cycles per pass and in the evaluation (dfmi_set_tuning("probe", 1) counters), and
the LM-only time against the one-segment-per-lane kernel, on config-2 QI (dfmi_demod,
component-major, guess [1, 6, 0, 0] like bench.py's lm_all_segments)."""
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
from deepfmkit_amd import fit as F  # noqa: E402
from deepfmkit_amd.fitters import w0_of  # noqa: E402

lib = _lib.load()
dev = torch.device("cuda", 0)
R, nd = 4000, 10
nseg = int(os.environ.get("NSEG", 100000))
st = torch.cuda.current_stream()
cfg = F.lm_config()
x = bench.gen_shard(torch, dev, 0, nseg, R, seed=bench.SEED)
qi = torch.empty((2 * nd, nseg), dtype=torch.float64, device=dev)
dc = torch.empty(nseg, dtype=torch.float64, device=dev)
_lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0_of(1000.0, 200000.0), 0, qi.data_ptr(), dc.data_ptr(), 1,
                          st.cuda_stream), "demod")
del x
g = torch.tensor([1.0, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
p = torch.empty((4, nseg), dtype=torch.float64, device=dev)
ssq = torch.empty(nseg, dtype=torch.float64, device=dev)
status = torch.empty(nseg, dtype=torch.int32, device=dev)


def lm():
    _lib.check(lib.dfmi_lm(qi.data_ptr(), nseg, nd, g.data_ptr(), 0, nseg, cfg, p.data_ptr(), ssq.data_ptr(),
                           status.data_ptr(), 1, st.cuda_stream), "lm")


def timed(n=20):
    lm()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(n):
        lm()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


settings = [dict(lm_refill=0), dict(lm_refill=1, lm_waves_per_simd=1, lm_tile_min=64),
            dict(lm_refill=1, lm_waves_per_simd=2, lm_tile_min=64)]
out = {}
ref = None
for s in settings:
    for k, v in s.items():
        _lib.check(lib.dfmi_set_tuning(k.encode(), v), k)
    ms = timed()
    cur = torch.cat([p.flatten(), ssq, status.double()]).cpu().numpy()
    if ref is None:
        ref = cur
    same = bool(np.array_equal(cur, ref))
    rec = {"ms": round(ms, 4), "bit_identical_to_first": same}
    if s.get("lm_refill"):
        _lib.check(lib.dfmi_set_tuning(b"probe", 0), "probe")
        _lib.check(lib.dfmi_set_tuning(b"probe", 1), "probe")
        lm()
        pr = (ctypes.c_int64 * 16)()
        _lib.check(lib.dfmi_probe_read(pr, 16), "probe_read")
        _lib.check(lib.dfmi_set_tuning(b"probe", 0), "probe")
        passes, busy, cyc, waves, tev, tsv, tdn, tst = (pr[i] for i in range(8, 16))
        rec.update({"waves": waves, "passes_per_wave": passes / waves, "busy_lanes_per_pass": busy / max(passes, 1),
                    "lane_passes_per_segment": busy / nseg, "cycles_per_wave": cyc / waves,
                    "cycles_per_pass": cyc / max(passes, 1), "eval_cycles_per_pass": tev / max(passes, 1),
                    "solve_cycles_per_pass": tsv / max(passes, 1), "done_cycles_per_pass": tdn / max(passes, 1),
                    "stage_cycles_per_wave": tst / waves})
    out[",".join(f"{k}={v}" for k, v in s.items())] = rec
    print(json.dumps({list(out)[-1]: rec}), flush=True)
