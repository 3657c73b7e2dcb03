"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE — separate runs) of one
kernel into profiles/pmc_demod.json, the file bench.py reads for roofline.traffic.

Usage: python scripts/pmc_summary.py <fetch_dir> <write_dir> <kernel-substring> <algorithmic_bytes_per_launch> <cmd>
The gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE
counts half the bytes of 16-B/lane streaming loads -> x2; WRITE_SIZE is exact.
"""
import collections
import csv
import glob
import json
import os
import sys


def counter_rows(d, counter, kernel_sub):
    """The counter per launch of the kernel, over the launches of the step's own grid (the most
    frequent one: bench.py's scaling_anchor runs the same kernel over 12.5x the segments)."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per, name = {}, None
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == counter and kernel_sub in r["Kernel_Name"]:
                    key = (f, r["Dispatch_Id"])
                    v, _ = per.get(key, (0.0, None))
                    per[key] = (v + float(r["Counter_Value"]), r["Grid_Size"])
                    name = r["Kernel_Name"]
    if not per:
        raise SystemExit(f"no {counter} rows for {kernel_sub} in {d}")
    grids = collections.Counter(g for _, g in per.values())
    grid = grids.most_common(1)[0][0]
    return name, [v for v, g in per.values() if g == grid], grid, len(per)


def main():
    fetch_dir, write_dir, sub, algo, cmd = sys.argv[1:6]
    name, fetch, grid, n_all = counter_rows(fetch_dir, "FETCH_SIZE", sub)
    _, write, _, _ = counter_rows(write_dir, "WRITE_SIZE", sub)
    f_kb = sum(fetch) / len(fetch)
    w_kb = sum(write) / len(write)
    hbm = (2 * f_kb + w_kb) * 1024
    algo = float(algo)
    out = {"kernel": name, "launches": len(fetch), "grid": grid, "launches_other_grids": n_all - len(fetch),
           "command": cmd,
           "FETCH_SIZE_kB_per_launch": f_kb, "WRITE_SIZE_kB_per_launch": w_kb,
           "correction": "gfx950: FETCH_SIZE counts half the bytes of 16-B/lane streaming loads "
                         "(MI355X_MICROARCH.md HBM section) -> x2; WRITE_SIZE exact",
           "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": algo,
           "traffic_over_algorithmic": hbm / algo,
           "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes: {fetch_dir}, {write_dir}"}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "profiles", "pmc_demod.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
