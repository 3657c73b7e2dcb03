"""CPU-baseline proxy check: time the oracle restatement of
StandardNLSFitter._fit_parallel (oracle/nls_oracle.py fit_record_parallel, numpy +
multiprocessing.Pool) beside the REAL reference's _fit_parallel (fitters.py:395-428,
imported read-only from /root/reference) on the same 10,000-segment config-2 input, in
this container (the reference never travels to the GPU box), and record the ratio:
bench.py's cpu_baseline on the GPU box times the restatement, so the ratio says how
faithfully it stands in for the reference there.

Writes profiles/r02_cpu_ratio.json. Usage: python scripts/ratio_vs_reference.py [nseg]
"""
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    from make_golden import _import_reference
    rdfm, _, rfitters = _import_reference()
    import DeepFMKit.physics as rphys
    from DeepFMKit.helpers import set_laser_df_for_effect

    from oracle import nls_oracle as O

    nseg = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    f_samp, f_mod, n, R = 200000.0, 1000.0, 20, 4000
    laser = rphys.LaserConfig()
    ifo = rphys.InterferometerConfig()
    set_laser_df_for_effect(laser, ifo, 6.0)
    sim = rphys.DFMIObject("ratio", laser, ifo, f_samp=f_samp)
    dff = rdfm.DeepFitFramework()
    dff.sims["ratio"] = sim
    dff.simulate("ratio", n_seconds=nseg * R / f_samp, mode="snr", snr_db=40.0, trial_num=0)
    raw = dff.raws["ratio"]
    x = np.asarray(raw.data["ch0"].to_numpy(), dtype=np.float64)
    cores = os.cpu_count()

    t0 = time.perf_counter()
    ref_df = rfitters.StandardNLSFitter({"n": n}).fit(raw, parallel=True)  # Pool(os.cpu_count())
    t_ref = time.perf_counter() - t0
    t0 = time.perf_counter()
    ours = O.fit_record_parallel(x, f_samp, f_mod, n, n_cores=cores)
    t_or = time.perf_counter() - t0
    cols = ["amp", "m", "phi", "psi", "dc", "ssq", "fitok"]
    same = all(np.array_equal(ref_df[c].to_numpy(dtype=np.float64), ours[:, i]) for i, c in enumerate(cols))
    out = {"segments": nseg, "cores": cores, "cpu_model": cpu_model(),
           "reference_fit_parallel": {"seconds": round(t_ref, 3), "segments_per_s": round(nseg / t_ref, 1)},
           "oracle_fit_record_parallel": {"seconds": round(t_or, 3), "segments_per_s": round(nseg / t_or, 1)},
           "ratio_oracle_over_reference": round(t_ref / t_or, 3),
           "results_bit_identical": bool(same),
           "input": "config 2 shape: snr-mode m=6, 40 dB, R=4000, RandomState(0) (the reference's own generator)",
           "where": "this build container (the reference is not on the GPU box)"}
    print(json.dumps(out, indent=1))
    with open(os.path.join(ROOT, "profiles", "r02_cpu_ratio.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
