"""PMC helper: one dfmi_lm launch per LM kernel variant (lm_general 0 / 1) over config-2
QI, for `rocprofv3 --pmc ...` per-dispatch counters (dynamic instruction counts).
Env: NSEG (100000), ND (10: harmonics), M (6.0: the record's m), SETTINGS (tuning sets,
';'-separated, each 'key=value,key=value'), GUESS_M (the LM's seed m, default M)."""
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
R, nd, nseg = 4000, int(os.environ.get("ND", 10)), int(os.environ.get("NSEG", 100000))
m_true = float(os.environ.get("M", 6.0))
st = torch.cuda.current_stream()
x = bench.gen_shard(torch, dev, 0, nseg, R, seed=bench.SEED, m_true=m_true)
qi = torch.empty((2 * nd, nseg), dtype=torch.float64, device=dev)
dc = torch.empty(nseg, dtype=torch.float64, device=dev)
_lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0_of(1000.0, 200000.0), 0, qi.data_ptr(), dc.data_ptr(), 1,
                          st.cuda_stream), "demod")
del x
g = torch.tensor([1.0, float(os.environ.get("GUESS_M", m_true)), 0.0, 0.0], dtype=torch.float64, device=dev)
p = torch.empty((4, nseg), dtype=torch.float64, device=dev)
ssq = torch.empty(nseg, dtype=torch.float64, device=dev)
status = torch.empty(nseg, dtype=torch.int32, device=dev)
cfg = F.lm_config()
for spec in os.environ.get("SETTINGS", "lm_general=0;lm_general=1").split(";"):
    for kv in filter(None, spec.split(",")):
        k, v = kv.split("=")
        _lib.check(lib.dfmi_set_tuning(k.encode(), int(v)), k)
    _lib.check(lib.dfmi_lm(qi.data_ptr(), nseg, nd, g.data_ptr(), 0, nseg, cfg, p.data_ptr(), ssq.data_ptr(),
                           status.data_ptr(), 1, st.cuda_stream), "lm")
    torch.cuda.synchronize()
print("ok")
