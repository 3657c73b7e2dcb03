"""Where a witness-fitter evaluation spends its time: dfmi_set_tuning("probe", 1)
makes workgroup 0 / thread 0 accumulate s_memrealtime ticks (10 ns) per phase:
[0] buffer load + mean, [1] cost evaluations, [5] optimiser scalar code and
harmonic sums between evaluations, [7] evaluation count."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.argv += [] 
from deepfmkit_amd import _lib  # noqa: E402
from scripts.bench_wdfmi import C_LIGHT  # noqa: E402
from deepfmkit_amd import fitters as F  # noqa: E402

G = np.load(os.path.join(ROOT, "tests", "golden", "wdfmi.npz"))
cases = {c["name"]: c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "wdfmi_cases.json")))["cases"]}
f_samp, f_mod, df, meas, ref, f_ref, n = G["cos_cfg"]
R = 4000
main = G["cos_main"][: 3 * R]
lib = _lib.load()
_lib.check(lib.dfmi_set_tuning(b"probe", 1), "probe")
for method, wit, kw in (("hwdfmi", G["cos_hw_witness"], dict(df=df, tau_init=(meas - ref) / C_LIGHT, f_ref=f_ref)),
                        ("wdfmi_ortho", G["cos_witness"], dict(df=df, tau_init=(meas - ref) / C_LIGHT, init_psi=0.3))):
    for _ in range(2):
        F.wdfmi_records(method, main[None], wit, f_samp, f_mod, R, 3, **kw)
    buf = (ctypes.c_int64 * 8)()
    _lib.check(lib.dfmi_probe_read(buf, 8), "probe_read")
    v = list(buf)
    names = ["load", "evaluate", "-", "-", "-", "between", "-", "evals"]
    us = {names[i]: v[i] / 100.0 for i in range(6)}
    print(json.dumps({"method": method, "buffers": 3, "evals": v[7], "us_total": us,
                      "us_per_eval": {k: round(x / max(v[7], 1), 2) for k, x in us.items()}}))
