"""Account bench.py's timed window from a rocprofv3 trace of the driver's command
(`rocprofv3 --kernel-trace --marker-trace --stats -- python3 bench.py --gpus 1 --steps 20
--warmup 5`): the roctx range "timed_window" (bench.py roctx_push / roctx_pop) gives the host
window; the kernel trace inside it gives the kernels' sum, the lag from the window's start to
the first kernel, the gaps between kernels and the tail from the last kernel to the window's
end (the final synchronize). One JSON object.

usage: python scripts/window_check.py TRACE_DIR STEPS
"""
import csv
import glob
import json
import os
import sys


def rows(pattern):
    out = []
    for f in sorted(glob.glob(pattern, recursive=True)):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main():
    d, steps = sys.argv[1], int(sys.argv[2])
    marks = [r for r in rows(os.path.join(d, "**", "*marker_api_trace.csv")) if "timed_window" in json.dumps(r)]
    if not marks:
        print(json.dumps({"error": "no timed_window marker in " + d}))
        return 1
    m = marks[-1]
    w0, w1 = int(m["Start_Timestamp"]), int(m["End_Timestamp"])
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in rows(os.path.join(d, "**", "*kernel_trace.csv")))
    inside = [k for k in ks if w0 <= k[0] <= w1]
    if not inside:
        print(json.dumps({"error": "no kernels inside the window"}))
        return 1
    busy = sum(e - s for s, e, _ in inside)
    gaps = [inside[i + 1][0] - inside[i][1] for i in range(len(inside) - 1)]
    by = {}
    for s, e, n in inside:
        key = n.split("(")[0]
        by[key] = by.get(key, 0) + (e - s)
    out = {
        "window_ms": (w1 - w0) / 1e6, "steps": steps, "window_ms_per_step": (w1 - w0) / 1e6 / steps,
        "kernels": len(inside), "kernels_ms_per_step": busy / 1e6 / steps,
        "first_launch_lag_us": (inside[0][0] - w0) / 1e3,
        "gaps_us_per_step": sum(gaps) / 1e3 / steps, "max_gap_us": max(gaps) / 1e3 if gaps else 0.0,
        "tail_us": (w1 - inside[-1][1]) / 1e3,
        "kernel_ms_per_step": {k: round(v / 1e6 / steps, 4) for k, v in sorted(by.items(), key=lambda kv: -kv[1])},
    }
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
