"""Per-record parity report of the GPU NLS path against the golden fixtures (the
numbers behind tests/test_gpu_parity.py::test_records_through_fitter): max |d amp|,
|d m|, wrapped |d phi|, |d psi| over status-0 segments, status match, per mode."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import make_record, wrapped  # noqa: E402

from deepfmkit_amd.fitters import StandardNLSFitter  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
man = json.load(open(os.path.join(G, "manifest.json")))
npz = np.load(os.path.join(G, "records.npz"))
out = []
for e in man["records"]:
    if e["name"] == "ragged_tail":
        continue
    raw = make_record(e).raws[e["name"]]
    for mode in ("seq", "c1", "par4"):
        if f"{e['name']}_{mode}_amp" not in npz.files:
            continue
        kw = dict(ndata=e["ndata"], init_m=e["init_m"])
        if mode == "seq":
            df = StandardNLSFitter({"n": e["n"]}).fit(raw, parallel=False, **kw)
        elif mode == "c1":
            df = StandardNLSFitter({"n": e["n"]}).fit(raw, parallel=True, **kw)
        else:
            df = StandardNLSFitter({"n": e["n"]}).fit(raw, parallel=True, n_cores=4, **kw)
        ref = {k: npz[f"{e['name']}_{mode}_{k}"] for k in ("amp", "m", "phi", "psi", "fitok")}
        st = df["fitok"].to_numpy()
        ok = (st == ref["fitok"]) & (st == 0)
        rec = {"record": e["name"], "mode": mode, "n": int(st.size), "status_match": float(np.mean(st == ref["fitok"]))}
        for k in ("amp", "m", "psi"):
            d = np.abs(df[k].to_numpy() - ref[k])[ok]
            rec[k] = float(d.max()) if d.size else None
            if d.size:
                rec[k + "_argmax"] = int(np.where(ok)[0][np.argmax(d)])
        d = wrapped(df["phi"].to_numpy() - ref["phi"])[ok]
        rec["phi"] = float(d.max()) if d.size else None
        out.append(rec)
        print(json.dumps(rec), flush=True)
