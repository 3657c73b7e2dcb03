"""GPU diagnostic: the witness fitters (dfmi_wdfmi_fit) against the reference's own
outputs in tests/golden/wdfmi.npz, per case and method, with timings."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from deepfmkit_amd import fitters as F  # noqa: E402

G = np.load(os.path.join(ROOT, "tests", "golden", "wdfmi.npz"))
CASES = {c["name"]: c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "wdfmi_cases.json")))["cases"]}
COLS = ["amp", "m", "phi", "psi", "tau", "dc", "ssq"]
C = 299792458.0


def run(case, method, reps=1, period=0):
    f_samp, f_mod, df, meas, ref, f_ref, n = G[f"{case}_cfg"]
    c = CASES[case]
    R = int(f_samp / f_mod * int(n))
    main = G[f"{case}_main"]
    nbuf = len(main) // R
    dl = meas - ref
    kw = dict(df=df, period=period)
    if method == "wdfmi_nls":
        wit = G[f"{case}_witness"]
        kw.update(tau_init=dl / C, init_a=c["nls"]["init_a"], init_phi=c["nls"]["init_phi"],
                  init_psi=c["nls"]["init_psi"])
    elif method in ("wdfmi_ortho", "wdfmi_seq"):
        wit = G[f"{case}_witness"]
        kw.update(tau_init=dl / C if df > 0 else 0.0, init_psi=c["ortho" if method == "wdfmi_ortho" else "seq"]["init_psi"])
    else:
        wit = G[f"{case}_hw_witness"]
        kw.update(tau_init=dl / C, f_ref=f_ref)
    mains = np.stack([main[: nbuf * R]] * reps)
    t0 = time.time()
    cols, ok = F.wdfmi_records(method, mains, wit, f_samp, f_mod, R, nbuf, **kw)
    dt = time.time() - t0
    return cols, ok, nbuf, dt


if __name__ == "__main__":
    for case in ("cos", "dist"):
        for method in ("wdfmi_ortho", "hwdfmi", "wdfmi_seq", "wdfmi_nls"):
            cols, ok, nbuf, dt = run(case, method)
            dev = {}
            for i, k in enumerate(COLS):
                ref = G[f"{case}_{method}_{k}"]
                dev[k] = float(np.max(np.abs(cols[i][:nbuf] - ref) / np.maximum(np.abs(ref), 1e-300)))
            okm = bool(np.all(ok[:nbuf] == G[f"{case}_{method}_fitok"]))
            print(json.dumps({"case": case, "method": method, "nbuf": nbuf, "s": round(dt, 4), "fitok_match": okm,
                              "rel": dev, "gpu_tau": cols[4][:nbuf].tolist(), "ref_tau": G[f"{case}_{method}_tau"].tolist()}),
                  flush=True)
    # throughput: many records in one call
    for method in ("wdfmi_ortho", "hwdfmi", "wdfmi_seq", "wdfmi_nls"):
        cols, ok, nbuf, dt = run("cos", method, reps=256)
        cols, ok, nbuf, dt = run("cos", method, reps=256)
        print(json.dumps({"method": method, "records": 256, "buffers": 256 * nbuf, "s": round(dt, 4),
                          "buffers_per_s": 256 * nbuf / dt}), flush=True)
