"""Where the facade's time goes (config 2, device-resident record): cProfile of
DeepFitFramework.fit(label, n=20) on a 100,000-segment record already on the GPU, plus
the same call's pieces timed by hand (the engine call alone, the D2H, the DataFrame /
DeepFitObject). One JSON line + the cProfile table on stderr."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import deepfmkit_amd as dfm
    from deepfmkit_amd.fitters import nls_records, frame_from
    dev = torch.device("cuda", 0)
    R, nseg = 4000, 100_000
    x = bench.gen_shard(torch, dev, 0, nseg, R, seed=bench.SEED)
    raw = dfm.DeepRawObject(x)
    raw.f_samp, raw.f_mod, raw.label = 200000.0, 1000.0, "c2"
    dff = dfm.DeepFitFramework()
    dff.raws["c2"] = raw
    for _ in range(2):
        dff.fit("c2", n=20, fit_label="e2e")
    torch.cuda.synchronize()
    res = {}
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        dff.fit("c2", n=20, fit_label="e2e")
        ts.append(time.perf_counter() - t0)
    res["facade_ms"] = round(float(np.median(ts)) * 1e3, 3)
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cols, ok = nls_records(x.reshape(1, -1), 200000.0, 1000.0, R, nseg)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        c, o = cols.cpu().numpy(), ok.cpu().numpy()
        t2 = time.perf_counter()
        df = frame_from(c, o)
        t3 = time.perf_counter()
        ts.append((t1 - t0, t2 - t1, t3 - t2))
    ts = np.median(np.array(ts), axis=0)
    res.update(engine_ms=round(ts[0] * 1e3, 3), d2h_ms=round(ts[1] * 1e3, 3), frame_ms=round(ts[2] * 1e3, 3))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        dff.fit("c2", n=20, fit_label="e2e")
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(30)
    print(s.getvalue(), file=sys.stderr)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
