"""Recompute the bench line's roofline fraction from a rocprofv3 kernel trace of the same
command (scripts/profile_round.sh): the step's dominant kernel's launches in
<trace>/bench_kernel_trace.csv, their mean / median duration, the fraction each gives
with the line's algorithmic bytes and peak, and the relative difference to the line's
event-timed avg_launch_ms. Usage: frac_check.py <bench_line.json> <kernel_trace.csv>"""
import collections
import csv
import json
import statistics
import sys


def main():
    line = json.load(open(sys.argv[1]))
    roof = line["roofline"]
    name = roof["kernel"].split("<")[0]
    rows = [r for r in csv.DictReader(open(sys.argv[2])) if name in r["Kernel_Name"]]
    # the main workload's launches only: the extra configs (two channels, the 1.25M-segment
    # shard, ...) launch the same kernel over other grids; keep the most frequent grid
    grids = collections.Counter(r.get("Grid_Size_X", "") for r in rows)
    main_grid = grids.most_common(1)[0][0] if grids else ""
    rows = [r for r in rows if r.get("Grid_Size_X", "") == main_grid]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6 for r in rows]  # ms
    B, peak = roof["algorithmic_bytes_per_launch"], roof["peak"]

    def frac(ms):
        return B / (ms * 1e-3) / 1e9 / peak

    mean, med = statistics.mean(d), statistics.median(d)
    out = {"kernel": rows[0]["Kernel_Name"] if rows else name, "launches": len(d), "grid_x": main_grid,
           "trace_mean_ms": round(mean, 5), "trace_median_ms": round(med, 5), "trace_min_ms": round(min(d), 5),
           "line_avg_launch_ms": roof["avg_launch_ms"], "line_frac": roof["frac"],
           "frac_from_trace_mean": round(frac(mean), 4), "frac_from_trace_median": round(frac(med), 4),
           "rel_diff_mean_vs_line": round(frac(mean) / roof["frac"] - 1.0, 4),
           "note": "the line times the kernel with HIP events around its launch (dispatch included); the trace "
                   "mean also holds the run's first, clock-ramp launches"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
