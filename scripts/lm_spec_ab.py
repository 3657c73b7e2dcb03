"""LM-only time (dfmi_lm over config-2 QI, chunk size 1) in the three descent modes of
the knob lm_spec (0 split trial / accept, 1 speculative ladder, 2 fused evaluation, 3 QI in registers), interleaved in one process, at 1 024 / 65 536 / 100 000
segments (guess [1, 6, 0, 0] as in scripts/lm_variant_ab.py, and the record seed)."""
import json
import os
import sys

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
st = torch.cuda.current_stream()
xall = bench.gen_shard(torch, dev, 0, 100000, R, seed=bench.SEED)
res = {}
for nseg in (1024, 65536, 100000):
    qi = torch.empty((2 * nd, nseg), dtype=torch.float64, device=dev)
    dc = torch.empty(nseg, dtype=torch.float64, device=dev)
    _lib.check(lib.dfmi_demod(xall.data_ptr(), nseg, R, R, nd, w0_of(1000.0, 200000.0), 0, qi.data_ptr(),
                              dc.data_ptr(), 1, st.cuda_stream), "demod")
    for gname, gv in (("g1600", [1.6, 6.0, 0.0, 0.0]), ("g1000", [1.0, 6.0, 0.0, 0.0])):
        g = torch.tensor(gv, dtype=torch.float64, device=dev)
        p = torch.empty((4, nseg), dtype=torch.float64, device=dev)
        ssq = torch.empty(nseg, dtype=torch.float64, device=dev)
        status = torch.empty(nseg, dtype=torch.int32, device=dev)

        def lm():
            _lib.check(lib.dfmi_lm(qi.data_ptr(), nseg, nd, g.data_ptr(), 0, nseg, F.lm_config(), p.data_ptr(),
                                   ssq.data_ptr(), status.data_ptr(), 1, st.cuda_stream), "lm")
        for rep in range(3):
            for spec in (0, 1, 2, 3):
                _lib.check(lib.dfmi_set_tuning(b"lm_spec", spec), "tuning")
                lm()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(20):
                    lm()
                e1.record(st)
                torch.cuda.synchronize()
                res.setdefault(f"{nseg}_{gname}_spec{spec}", []).append(round(e0.elapsed_time(e1) / 20, 4))
_lib.check(lib.dfmi_set_tuning(b"lm_spec", 3), "tuning")
print(json.dumps(res), flush=True)
