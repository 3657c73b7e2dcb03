"""Probe: the many-harmonic step as a two-part pipeline (diagnostics).

Config 2 (100k segments, R = 4000) at ndata ND (62): the LM is ~0.2 ms after a ~0.59 ms
demodulation (demod_wide_kernel, component-major QI). Cut the segments at a fraction F:
  serial   demod(all) then lm(all), one stream
  pipe_F   stream A: demod(a), demod(b); stream B: lm(a) behind demod(a)'s event; then lm(b)
           behind both (the LM of part a in the slots demod(b) leaves)
  lm_a_F / lm_b_F   each LM part alone
Each part's QI goes to its own component-major buffer (its dfmi_demod call's layout). One JSON
line. env: ND (62), FRACS ("0.5,0.6,0.7,0.8")."""
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
    nseg, R, nd = 100000, 4000, int(os.environ.get("ND", 62))
    x = bench.gen_shard(torch, dev, 0, nseg, R, seed=bench.SEED)
    w0 = w0_of(1000.0, 200000.0)
    g = torch.tensor([1.0, 6.0, 0.0, 0.0], dtype=torch.float64, device=dev)
    cfg = F.lm_config()
    cur = torch.cuda.current_stream()

    class Part:
        def __init__(self, s0, n):
            self.s0, self.n = s0, n
            self.q = torch.empty((2 * nd, n), dtype=torch.float64, device=dev)
            self.dc = torch.empty(n, dtype=torch.float64, device=dev)
            self.p = torch.empty((4, n), dtype=torch.float64, device=dev)
            self.ssq = torch.empty(n, dtype=torch.float64, device=dev)
            self.st = torch.empty(n, dtype=torch.int32, device=dev)

        def demod(self, s):
            _lib.check(lib.dfmi_demod(x.data_ptr() + self.s0 * R * 8, self.n, R, R, nd, w0, 0, self.q.data_ptr(),
                                      self.dc.data_ptr(), 1, s.cuda_stream), "demod")

        def lm(self, s):
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

    whole = Part(0, nseg)
    for _ in range(20):  # clock ramp
        whole.demod(cur)
    res = {"nseg": nseg, "ndata": nd}
    res["serial"] = timed(lambda: (whole.demod(cur), whole.lm(cur)))
    res["demod"] = timed(lambda: whole.demod(cur))
    res["lm"] = timed(lambda: whole.lm(cur))
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    for frac in [float(v) for v in os.environ.get("FRACS", "0.5,0.6,0.7,0.8").split(",")]:
        na = int(nseg * frac) // 64 * 64
        a, b = Part(0, na), Part(na, nseg - na)
        ev0, eva, evb, evl = torch.cuda.Event(), torch.cuda.Event(), torch.cuda.Event(), torch.cuda.Event()

        def pipe():
            ev0.record(cur)
            sa.wait_event(ev0)
            sb.wait_event(ev0)
            a.demod(sa)
            eva.record(sa)
            b.demod(sa)
            sb.wait_event(eva)
            a.lm(sb)
            evl.record(sb)
            sa.wait_event(evl)
            b.lm(sa)
            evb.record(sa)
            cur.wait_event(evb)

        res[f"pipe_{frac}"] = timed(pipe)
        res[f"lm_a_{frac}"] = timed(lambda: a.lm(cur))
        res[f"lm_b_{frac}"] = timed(lambda: b.lm(cur))
        del a, b
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
