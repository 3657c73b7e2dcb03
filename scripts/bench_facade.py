"""End-to-end time of the drop-in facade on the reference's own benchmark call
(notebooks/0.0_benchmark.ipynb cell 4: dff.fit(label, n=20, parallel=False)) and its parallel
form, config 1 (10 s @ 200 kS/s = 500 segments, m = 6, 40 dB), input in host memory as the
reference holds it (a pandas column): H2D, demodulation, LM, D2H and the DataFrame /
DeepFitObject construction included. Median of 20 calls after 3 warm-up calls. One JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import deepfmkit_amd as dfm
    laser, ifo = dfm.LaserConfig(), dfm.InterferometerConfig()
    dfm.set_laser_df_for_effect(laser, ifo, 6.0)
    dff = dfm.DeepFitFramework()
    dff.load_sim(dfm.DFMIObject("raw1", laser, ifo, f_samp=200000.0))
    dff.simulate("raw1", n_seconds=10.0, mode="snr", snr_db=40.0, trial_num=0)
    res = {}
    for name, kw in (("sequential", dict(parallel=False)), ("parallel", dict(parallel=True))):
        for _ in range(3):
            dff.fit("raw1", n=20, **kw)
        ts = []
        for _ in range(20):
            t0 = time.perf_counter()
            fo = dff.fit("raw1", n=20, **kw)
            ts.append(time.perf_counter() - t0)
        ms = float(np.median(ts)) * 1e3
        res[name] = {"ms_per_call": round(ms, 3), "segments": int(len(fo.m)), "segments_per_s": round(len(fo.m) / ms * 1e3, 1)}
    res["reference_same_calls"] = "724 (sequential) / 2,091 (parallel, 8 cores) segments/s, BASELINE.md"
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
