"""Throughput of the witness-based fitters (dfmi_wdfmi_fit) on the GPU, next to the
CPU oracle (the restated reference loop, one core), on the reference's own W-DFMI
inputs (tests/golden/wdfmi.npz 'cos' case: f_samp 200 kHz, f_mod 1 kHz, n = 20 ->
R = 4000, m = 6, witness m = 0.5).

A workload is `nrec` independent records (channels / trials) of `nbuf` buffers each,
resident in HBM; nls / ortho / hwdfmi chain their buffers (warm start, one workgroup
per record), seq fits every buffer independently (one workgroup per buffer). Timing:
HIP events on the launch stream around one dfmi_wdfmi_fit call (median of `reps`).

One JSON line per (method, nrec) on stdout.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

C_LIGHT = 299792458.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--methods", default="wdfmi_ortho,hwdfmi,wdfmi_seq,wdfmi_nls")
    ap.add_argument("--records", default="1,256,2048")
    ap.add_argument("--nbuf", type=int, default=9)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--cpu", type=int, default=1, help="time the oracle on one record (1 core)")
    ap.add_argument("--accel", default="", help="comma list of wdfmi_accel tuning values to compare (default: 3)")
    args = ap.parse_args()

    import torch

    from deepfmkit_amd import _lib
    from deepfmkit_amd import fitters as F

    G = np.load(os.path.join(ROOT, "tests", "golden", "wdfmi.npz"))
    cases = {c["name"]: c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "wdfmi_cases.json")))["cases"]}
    f_samp, f_mod, df, meas, ref, f_ref, n = G["cos_cfg"]
    c = cases["cos"]
    R = int(f_samp / f_mod * int(n))
    base = G["cos_main"]
    reps_needed = -(-args.nbuf * R // len(base))
    rec = np.tile(base, reps_needed)[: args.nbuf * R]
    dl = meas - ref
    dev = torch.device("cuda:0")
    for method in args.methods.split(","):
        if method == "hwdfmi":
            wit = G["cos_hw_witness"]
            kw = dict(df=df, tau_init=dl / C_LIGHT, f_ref=f_ref)
        elif method == "wdfmi_nls":
            wit = G["cos_witness"]
            kw = dict(df=df, tau_init=dl / C_LIGHT, **c["nls"])
        else:
            wit = G["cos_witness"]
            kw = dict(df=df, tau_init=dl / C_LIGHT, **c["ortho" if method == "wdfmi_ortho" else "seq"])
        cpu = None
        if args.cpu:
            from oracle import wdfmi_oracle as W
            t0 = time.perf_counter()
            nb = 3
            if method == "wdfmi_nls":
                W.fit_wdfmi_nls(rec[: nb * R], wit, f_samp, f_mod, df, dl, int(n), **c["nls"])
            elif method == "wdfmi_ortho":
                W.fit_wdfmi_ortho(rec[: nb * R], wit, f_samp, f_mod, df, dl, int(n), **c["ortho"])
            elif method == "wdfmi_seq":
                W.fit_wdfmi_seq(rec[: nb * R], wit, f_samp, f_mod, df, dl, int(n), **c["seq"])
            else:
                W.fit_hwdfmi(rec[: nb * R], wit, f_samp, f_mod, f_ref, dl, int(n))
            cpu = {"value": nb / (time.perf_counter() - t0), "unit": "buffers/s", "cores": 1, "kind": "port",
                   "sample": f"{nb} buffers, oracle restatement of the reference loop (numpy/scipy algorithms)"}
        for nrec, acc in [(int(v), t) for v in args.records.split(",") for t in (args.accel.split(",") if args.accel else [""])]:
            _lib.check(_lib.load().dfmi_set_tuning(b"wdfmi_accel", int(acc) if acc else 3), "dfmi_set_tuning")
            x = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(rec, (nrec, rec.size)))).to(dev)
            w = torch.from_numpy(np.ascontiguousarray(wit[:R])).to(dev)
            F.wdfmi_records(method, x, w, f_samp, f_mod, R, args.nbuf, **kw)  # warm-up (tables, code objects)
            torch.cuda.synchronize()
            st = torch.cuda.current_stream()
            times = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                cols, ok = F.wdfmi_records(method, x, w, f_samp, f_mod, R, args.nbuf, **kw)
                e1.record(st)
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1) / 1e3)
            t = float(np.median(times))
            nb_tot = nrec * args.nbuf
            line = {"metric": "W-DFMI buffers fitted/sec", "method": method, "value": nb_tot / t, "unit": "buffers/s",
                    "records": nrec, "accel": int(acc) if acc else 3, "nbuf": args.nbuf, "R": R, "seconds": t,
                    "per_buffer_latency_ms": (t / args.nbuf if method != "wdfmi_seq" else t) * 1e3,
                    "fitok_frac": float(ok.float().mean().item()), "cpu_baseline": cpu,
                    "data": "reference W-DFMI 'cos' case (tests/golden/wdfmi.npz) tiled to nbuf buffers"}
            print(json.dumps(line), flush=True)
            del x


if __name__ == "__main__":
    main()
