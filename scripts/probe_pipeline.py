"""Probe: a two-part pipeline of the record step (diagnostics, DESIGN.md §4 "LM overlap").

Config-2 shapes (100k segments, R = 4000, ndata 10). The demodulation is cut at a
fraction F of the segments: part a = [0, F·N), part b = [F·N, N).
  serial      demod(all) then lm(all), one stream (what the step does today)
  pipe_F      stream A: demod(a), demod(b); stream B: lm(a) behind demod(a)'s event
              (it fills the slots demod(b) and the demodulation's tail leave free);
              then lm(b) behind both. lm(b) runs the lambda-ladder kernel when its
              segment count is at most lm_ladder x CUs (LADDER env, default 64)
  lm_b_F      lm(b) alone, both kernels (ladder / one lane per segment)
Inputs of the LM are component-major QI demodulated beforehand (the dependency is
reproduced by the events; the bytes the LM reads are the same size either way).
One JSON line."""
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
    nseg, R, nd = 100000, 4000, 10
    x = bench.gen_shard(torch, dev, 0, nseg, R, seed=1)
    w0 = w0_of(1000.0, 200000.0)
    qs = lib.dfmi_qi_row_stride(nd)
    rows = torch.empty((nseg, qs), dtype=torch.float64, device=dev)
    qi = torch.empty((2 * nd, nseg), dtype=torch.float64, device=dev)
    dc = torch.empty(nseg, dtype=torch.float64, device=dev)
    cur = torch.cuda.current_stream()
    _lib.check(lib.dfmi_demod(x.data_ptr(), nseg, R, R, nd, w0, 0, qi.data_ptr(), dc.data_ptr(), 1, cur.cuda_stream),
               "demod")
    g = torch.tensor([1.0, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    cfg = F.lm_config()
    ladder = int(os.environ.get("LADDER", 64))
    lib.dfmi_set_tuning(b"lm_ladder", ladder)

    def demod(s0, n, s):
        _lib.check(lib.dfmi_demod_rows(x.data_ptr() + s0 * R * 8, n, R, R, nd, w0, 0, rows.data_ptr() + s0 * qs * 8, 1,
                                       s.cuda_stream), "demod_rows")

    class LM:
        def __init__(self, s0, n):
            self.q = qi[:, s0:s0 + n].contiguous()
            self.n = n
            self.p = torch.empty((4, n), dtype=torch.float64, device=dev)
            self.ssq = torch.empty(n, dtype=torch.float64, device=dev)
            self.st = torch.empty(n, dtype=torch.int32, device=dev)

        def __call__(self, s):
            _lib.check(lib.dfmi_lm(self.q.data_ptr(), self.n, nd, g.data_ptr(), 0, self.n, cfg, self.p.data_ptr(),
                                   self.ssq.data_ptr(), self.st.data_ptr(), 1, s.cuda_stream), "lm")

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
        return round(float(np.median(out)), 5)

    lm_all = LM(0, nseg)
    for _ in range(30):  # clock ramp
        demod(0, nseg, cur)
    res = {"nseg": nseg, "ladder": ladder}
    res["serial"] = timed(lambda: (demod(0, nseg, cur), lm_all(cur)))
    res["demod"] = timed(lambda: demod(0, nseg, cur))
    res["lm"] = timed(lambda: lm_all(cur))
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for frac in (0.8, 0.9, 0.95, 0.98):
        na = int(nseg * frac) // 64 * 64
        nb = nseg - na
        lm_a, lm_b = LM(0, na), LM(na, nb)
        ev0, eva, evb, evl = torch.cuda.Event(), torch.cuda.Event(), torch.cuda.Event(), torch.cuda.Event()

        def pipe():
            ev0.record(cur)
            sa.wait_event(ev0)
            sb.wait_event(ev0)
            demod(0, na, sa)
            eva.record(sa)
            demod(na, nb, sa)
            sb.wait_event(eva)
            lm_a(sb)
            evl.record(sb)
            sa.wait_event(evl)
            lm_b(sa)
            evb.record(sa)
            cur.wait_event(evb)

        res[f"pipe_{frac}"] = timed(pipe)
        res[f"lm_b_{frac}"] = timed(lambda: lm_b(cur))
        lib.dfmi_set_tuning(b"lm_ladder", 0)
        res[f"lm_b_{frac}_noladder"] = timed(lambda: lm_b(cur))
        res[f"pipe_{frac}_noladder"] = timed(pipe)
        lib.dfmi_set_tuning(b"lm_ladder", ladder)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
