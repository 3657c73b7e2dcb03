"""Probe: can the LM kernel run beside the bulk demodulation without slowing it?

Config-2 shapes (100k segments, R = 4000, ndata 10). Times, with HIP events on a
join stream:
  demod      dfmi_demod_rows alone (the record pipeline's demodulation)
  lm         dfmi_lm alone over component-major QI of the same segments
  serial     demod then lm on one stream
  conc_*     demod on stream A and lm on stream B launched together (B waits only on
             the start event), for several (A, B) stream priorities: whether the
             dispatcher serves the low-priority queue only once the high-priority
             queue has no workgroups left (the LM then fills the demodulation's drain).
Prints one JSON line. Diagnostics only (LM overlap)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from deepfmkit_amd import _lib
    from deepfmkit_amd import fit as F
    from deepfmkit_amd.fitters import w0_of
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    nseg, R, nd = int(os.environ.get("NSEG", 100000)), 4000, 10
    frac = float(os.environ.get("LM_FRAC", 1.0))  # share of the segments the LM fits
    x = bench.gen_shard(torch, dev, 0, nseg, R, seed=1)
    w0 = w0_of(1000.0, 200000.0)
    qs = lib.dfmi_qi_row_stride(nd)
    rows = torch.empty((nseg, qs), dtype=torch.float64, device=dev)
    qi = torch.empty((2 * nd, nseg), dtype=torch.float64, device=dev)
    dc = torch.empty(nseg, dtype=torch.float64, device=dev)
    cur = torch.cuda.current_stream()
    _lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0, 0, qi.data_ptr(), dc.data_ptr(), 1, cur.cuda_stream),
               "demod")
    nlm = int(nseg * frac)
    qlm = qi[:, :nlm].contiguous()
    g = torch.tensor([1.0, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    cfg = F.lm_config()
    p = torch.empty((4, nlm), dtype=torch.float64, device=dev)
    ssq = torch.empty(nlm, dtype=torch.float64, device=dev)
    st = torch.empty(nlm, dtype=torch.int32, device=dev)

    def demod(s):
        _lib.check(lib.dfmi_demod_rows(x.data_ptr(), nseg, R, R, nd, w0, 0, rows.data_ptr(), 1, s.cuda_stream),
                   "demod_rows")

    def lm(s):
        _lib.check(lib.dfmi_lm(qlm.data_ptr(), nlm, nd, g.data_ptr(), 0, nlm, cfg, p.data_ptr(), ssq.data_ptr(),
                               st.data_ptr(), 1, s.cuda_stream), "lm")

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        out = []
        for _ in range(reps):
            e0.record(cur)
            fn()
            e1.record(cur)
            e1.synchronize()
            out.append(e0.elapsed_time(e1))
        return float(np.median(out)), float(np.min(out))

    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    res = {"nseg": nseg, "lm_segments": nlm, "priority_range": [lo, hi]}
    for _ in range(30):  # clock ramp
        demod(cur)
    res["demod"] = timed(lambda: demod(cur))
    res["lm"] = timed(lambda: lm(cur))
    res["serial"] = timed(lambda: (demod(cur), lm(cur)))
    # (round 3 also tried the LM's AQL packet without the barrier bit, hipExtAnyOrderLaunch
    # on one stream: no effect on gfx950, 0.5376 vs 0.5380 ms: profiles/r03e_probe_anyorder.txt)
    for name, pa, pb in (("conc_same", 0, 0), ("conc_Ahi", -1, 0), ("conc_Blo", 0, 0), ("conc_Bhi", 0, -1)):
        sa = torch.cuda.Stream(priority=pa)
        sb = torch.cuda.Stream(priority=pb)
        ev = torch.cuda.Event()
        evb = torch.cuda.Event()

        def conc():
            ev.record(cur)
            sa.wait_event(ev)
            sb.wait_event(ev)
            demod(sa)
            lm(sb)
            evb.record(sb)
            eva = torch.cuda.Event()
            eva.record(sa)
            cur.wait_event(eva)
            cur.wait_event(evb)

        res[name] = timed(conc)
        # the demodulation alone on stream A, the LM alone on B, as launched here
        res[name + "_demod_alone"] = timed(lambda: (ev.record(cur), sa.wait_event(ev), demod(sa),
                                                    cur.wait_stream(sa)))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
