"""Print the dfmi kernel timeline of a rocprofv3 --kernel-trace CSV (analysis helper).
Usage: python scripts/timeline.py <kernel_trace.csv> [first N kernels]"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "dfmi" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 15
t0 = int(rows[0]["Start_Timestamp"]) if rows else 0
for r in rows[:n]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void dfmi::", "")
    print(f"{name[:58]:58s} start {(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f} us  end {(e - t0) / 1e3:9.1f}")
