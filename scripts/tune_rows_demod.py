"""Interleaved A/B of the roofline kernel (dfmi_demod_rows: the bin kernel in the row
layout, config 2) under tuning settings, with a bit-identity check of the rows.
Usage: SETTINGS="demod_spw=2;demod_spw=0" python scripts/tune_rows_demod.py"""
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
from tune_step import parse  # noqa: E402

torch.cuda.set_device(0)
lib = _lib.load()
dev = torch.device("cuda", 0)
nseg, R, nd = int(os.environ.get("NSEG", 100000)), 4000, 10
x = bench.gen_shard(torch, dev, 0, nseg, R, seed=bench.SEED)
st = torch.cuda.current_stream()
rows = torch.empty((nseg, lib.dfmi_qi_row_stride(nd)), dtype=torch.float64, device=dev)
settings = parse(os.environ.get("SETTINGS", "demod_spw=2;demod_spw=0"))
defaults = {}
for s in settings:
    for k in s:
        v = ctypes.c_int64()
        _lib.check(lib.dfmi_get_tuning(k.encode(), ctypes.byref(v)), k)
        defaults[k] = v.value


def apply(s):
    for k, v in {**defaults, **s}.items():
        _lib.check(lib.dfmi_set_tuning(k.encode(), v), k)


def demod():
    _lib.check(lib.dfmi_demod_rows(x.data_ptr(), nseg, R, R, nd, w0_of(1000.0, 200000.0), 0, rows.data_ptr(),
                                   _lib.DFMI_MEM_DEVICE, st.cuda_stream), "demod")


ref = None
names = {}
for i, s in enumerate(settings):
    apply(s)
    demod()
    torch.cuda.synchronize()
    names[i] = lib.dfmi_last_demod_kernel().decode()
    cur = rows.clone()
    if ref is None:
        ref = cur
    else:
        assert torch.equal(cur, ref), s
res = {i: [] for i in range(len(settings))}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(6):
    for i, s in enumerate(settings):
        apply(s)
        demod()
        e0.record(st)
        for _ in range(10):
            demod()
        e1.record(st)
        e1.synchronize()
        res[i].append(e0.elapsed_time(e1) / 10)
out = {}
for i, s in enumerate(settings):
    ms = float(np.median(res[i]))
    out[",".join(f"{k}={v}" for k, v in s.items()) or "default"] = {
        "kernel": names[i], "ms": round(ms, 4), "TBps": round(nseg * (8 * R + 8 * (2 * nd + 1)) / ms / 1e9, 3)}
print(json.dumps(out, indent=1))
