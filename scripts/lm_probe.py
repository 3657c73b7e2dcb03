"""Cycle split of the register-path LM (scripts/lm_probe.hip): per lane, s_memtime
cycles in solve / trial / accept and the pass count, for one wave alone and for a
full config-2 batch; QI of config-2 segments from dfmi_demod (component-major)."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from deepfmkit_amd import _lib  # noqa: E402
from deepfmkit_amd.fitters import w0_of  # noqa: E402

so = os.path.join(ROOT, "scripts", "lm_probe.so")
lib = _lib.load()
nseg, R = 100_000, 4000
x = bench.gen_shard(torch, "cuda", 0, nseg, R, seed=bench.SEED)
qi = torch.empty((20, nseg), dtype=torch.float64, device="cuda")
dc = torch.empty(nseg, dtype=torch.float64, device="cuda")
_lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, 10, w0_of(1000.0, 200000.0), 0, qi.data_ptr(), dc.data_ptr(), 1,
                          torch.cuda.current_stream().cuda_stream), "demod")
q = qi.cpu().numpy()
del x
pl = ctypes.CDLL(so)
pl.lm_probe.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                        ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
g = np.array([1.0, 6.0, 0.0, 0.0])
res = {}
for n in (64, 65536, 100_000):
    qn = np.ascontiguousarray(q[:, :n])
    p = np.zeros((n, 4))
    cyc = np.zeros((n, 8), np.uint64)
    ms = ctypes.c_double()
    assert pl.lm_probe(qn.ctypes.data, n, g.ctypes.data, p.ctypes.data, cyc.ctypes.data, 5, ctypes.byref(ms)) == 0
    c = cyc.astype(np.float64)
    w = c[: (n // 64) * 64].reshape(-1, 64, 8)
    wave_total = w[:, :, 0].max(1)
    res[n] = {"ms": round(ms.value, 4), "wave_cycles_mean": float(wave_total.mean()),
              "lane_solve": float(c[:, 1].mean()), "lane_trial": float(c[:, 2].mean()),
              "lane_accept": float(c[:, 3].mean()), "lane_passes": float(c[:, 4].mean()),
              "wave_max_passes": float(w[:, :, 4].max(1).mean()), "lane_accepts": float(c[:, 5].mean()),
              "per_pass_solve": float((c[:, 1] / c[:, 4]).mean()), "per_trial": float((c[:, 2] / (c[:, 4] + 1)).mean()),
              "per_accept": float((c[:, 3] / (c[:, 5] + 1)).mean())}
    print(json.dumps({n: res[n]}), flush=True)
