"""Where DeepFitFramework.fit(label, n=20)'s time goes at config 2 (100,000 segments x R=4000,
record already on the GPU): perf_counter marks at every stage of the NLS path
(deepfmkit_amd.fitters.MARKS: fit entry, fitter arguments, output allocation, engine enqueue,
the wait for the kernels, the D2H of the result columns, the DataFrame, tau, the column
arrays, the DeepFitObject), median over calls, next to the call's wall time with marks off.
One JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    import deepfmkit_amd as dfm
    from deepfmkit_amd import fitters
    dev = torch.device("cuda", 0)
    R, nseg = 4000, int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    x = bench.gen_shard(torch, dev, 0, nseg, R, seed=bench.SEED)
    raw = dfm.DeepRawObject(x)
    raw.f_samp, raw.f_mod, raw.label = 200000.0, 1000.0, "c2"
    dff = dfm.DeepFitFramework()
    dff.raws["c2"] = raw
    for _ in range(3):
        dff.fit("c2", n=20, fit_label="e2e")
    torch.cuda.synchronize()
    calls = 11
    wall = []
    for _ in range(calls):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dff.fit("c2", n=20, fit_label="e2e")
        wall.append(time.perf_counter() - t0)
    stages = []
    for _ in range(calls):
        torch.cuda.synchronize()
        fitters.MARKS = [("start", time.perf_counter())]
        dff.fit("c2", n=20, fit_label="e2e")
        m = fitters.MARKS
        fitters.MARKS = None
        stages.append([(m[i][0], m[i][1] - m[i - 1][1]) for i in range(1, len(m))] + [("total", m[-1][1] - m[0][1])])
    names = [n for n, _ in stages[0]]
    med = {n: round(float(np.median([dict(s)[n] for s in stages])) * 1e3, 4) for n in names}
    print(json.dumps({"workload": f"DeepFitFramework.fit(label, n=20), {nseg} segments x R={R}, device-resident record",
                      "ms_per_call_marks_off": round(float(np.median(wall)) * 1e3, 4),
                      "stage_ms_marks_on (time since the previous mark)": med,
                      "torch": torch.__version__, "calls": calls}), flush=True)


if __name__ == "__main__":
    main()
