"""Interleaved timing of the LM kernel variants on config-2 QI (HIP events)."""
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


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    nseg, R, nd = int(os.environ.get("NSEG", 100000)), 4000, 10
    x = bench.gen_shard(torch, dev, 0, nseg, R, seed=1)
    qi = torch.empty((2 * nd, nseg), dtype=torch.float64, device=dev)
    dc = torch.empty(nseg, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream()
    _lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0_of(1000.0, 200000.0), 0, qi.data_ptr(),
                              dc.data_ptr(), 1, st.cuda_stream), "demod")
    del x
    cfg = F.lm_config()
    g = torch.tensor([1.0, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    outs = {}
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {"register": [], "general": []}
    for rnd in range(5):
        for name, gen in (("register", 0), ("general", 1)):
            lib.dfmi_set_tuning(b"lm_general", gen)
            p = torch.empty((4, nseg), dtype=torch.float64, device=dev)
            s = torch.empty(nseg, dtype=torch.float64, device=dev)
            k = torch.empty(nseg, dtype=torch.int32, device=dev)
            ev0.record(st)
            for _ in range(3):
                _lib.check(lib.dfmi_lm(qi.data_ptr(), nseg, nd, g.data_ptr(), 0, nseg, cfg, p.data_ptr(),
                                       s.data_ptr(), k.data_ptr(), 1, st.cuda_stream), "lm")
            ev1.record(st)
            ev1.synchronize()
            res[name].append(ev0.elapsed_time(ev1) / 3)
            outs[name] = p.cpu().numpy()
    lib.dfmi_set_tuning(b"lm_general", 0)
    d = np.abs(outs["register"] - outs["general"]).max(axis=1)
    print(json.dumps({k: round(float(np.median(v)), 4) for k, v in res.items()} |
                     {"max_abs_diff_register_vs_general": d.tolist()}))


if __name__ == "__main__":
    main()
