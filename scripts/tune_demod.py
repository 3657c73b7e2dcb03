"""Interleaved A/B timing of demod-kernel variants (one process, HIP events on the
launch stream) plus torch read-bandwidth references. Usage: python scripts/tune_demod.py"""
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


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    lib = _lib.load()
    nseg, R, nd = int(os.environ.get("NSEG", 100000)), 4000, 10
    x = bench.gen_shard(torch, dev, 0, nseg, R, seed=1)
    qi = torch.empty((2 * nd, nseg), dtype=torch.float64, device=dev)
    dc = torch.empty(nseg, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream()
    w0 = w0_of(1000.0, 200000.0)
    # (demod_kernel, demod_spw): fold kernel vs bin kernel, grid sizing
    variants = [tuple(int(t) for t in v.split(",")) for v in os.environ.get(
        "VARIANTS", "0,2;1,2;1,0;1,3").split(";")]
    keys = ("demod_kernel", "demod_spw")
    res = {v: [] for v in variants}
    ref = {"torch_sum": [], "torch_copy": []}
    y = torch.empty_like(x)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    nbytes = nseg * (8 * R + 8 * (2 * nd + 1))
    for rnd in range(6):
        for v in variants:
            for k, val in zip(keys, v):
                _lib.check(lib.dfmi_set_tuning(k.encode(), val), "tune")
            _lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0, 0, qi.data_ptr(), dc.data_ptr(), 1,
                                      st.cuda_stream), "demod")
            ev0.record(st)
            for _ in range(5):
                lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0, 0, qi.data_ptr(), dc.data_ptr(), 1, st.cuda_stream)
            ev1.record(st)
            ev1.synchronize()
            res[v].append(ev0.elapsed_time(ev1) / 5)
        ev0.record(st)
        for _ in range(5):
            x.sum()
        ev1.record(st)
        ev1.synchronize()
        ref["torch_sum"].append(ev0.elapsed_time(ev1) / 5)
        ev0.record(st)
        for _ in range(5):
            y.copy_(x)
        ev1.record(st)
        ev1.synchronize()
        ref["torch_copy"].append(ev0.elapsed_time(ev1) / 5)
    # all variants must agree with the fold kernel (same fold order; contraction identical)
    qref = None
    for v in variants:
        for k, val in zip(keys, v):
            _lib.check(lib.dfmi_set_tuning(k.encode(), val), "tune")
        _lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0, 0, qi.data_ptr(), dc.data_ptr(), 1,
                                  st.cuda_stream), "demod")
        torch.cuda.synchronize()
        cur = torch.cat([qi.flatten(), dc])
        if qref is None:
            qref = cur.clone()
        else:
            d = (cur - qref).abs().max().item()
            kn = lib.dfmi_last_demod_kernel().decode()
            print(f"variant {v} = {kn}", file=sys.stderr)
            print(f"variant {v}: max|diff| vs fold = {d:.3e}", file=sys.stderr)
            assert d <= 1e-13, (v, d)
    out = {}
    for v, t in res.items():
        med = float(np.median(t))
        kname = {0: "fold", 1: "bins"}[v[0]]
        name = f"{kname}_loads{v[1]}_nt{v[2]}_bpc{v[3]}"
        out[name] = {"ms": round(med, 4), "GBps": round(nbytes / med / 1e6, 1)}
    out["torch_sum_read_GBps"] = round(x.numel() * 8 / np.median(ref["torch_sum"]) / 1e6, 1)
    out["torch_copy_rw_GBps"] = round(2 * x.numel() * 8 / np.median(ref["torch_copy"]) / 1e6, 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
