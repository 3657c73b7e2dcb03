"""Summary of scripts/gpu_lm_general_pmc.sh output: per ndata, the LM kernel's duration (kernel
trace) and its counters (SQ_* summed over the dispatch), with per-wave figures.
usage: python scripts/lm_pmc_summary.py gpurun_out/TAG/lmpmc"""
import collections
import csv
import os
import sys


def main():
    d = sys.argv[1]
    for nd in sorted(int(x[2:]) for x in os.listdir(d) if x.startswith("nd") and x[2:].isdigit()):
        base = os.path.join(d, f"nd{nd}")
        dur = {}
        for r in csv.DictReader(open(os.path.join(base, "trace", "lm_kernel_stats.csv"))):
            dur[r["Name"]] = float(r["AverageNs"]) / 1e3
        aggs = collections.defaultdict(lambda: collections.defaultdict(float))  # per LM kernel variant
        metas = {}
        for g in ("a", "b"):
            for r in csv.DictReader(open(os.path.join(base, g, "lm_counter_collection.csv"))):
                if "lm_chunks_kernel" in r["Kernel_Name"]:
                    name = r["Kernel_Name"].split("(")[0]
                    aggs[name][r["Counter_Name"]] += float(r["Counter_Value"])
                    metas[name] = {"VGPR": r["VGPR_Count"], "AGPR": r["Accum_VGPR_Count"],
                                   "LDS": r["LDS_Block_Size"], "scratch": r["Scratch_Size"]}
        for name, agg in aggs.items():
            meta = metas[name]
            waves = agg.get("SQ_WAVES", 1.0)
            us = [v for k, v in dur.items() if k.split("(")[0] == name]
            print(f"ndata {nd}: {name} VGPR {meta.get('VGPR')} AGPR {meta.get('AGPR')} LDS "
                  f"{meta.get('LDS')} scratch {meta.get('scratch')}; duration {us[0] if us else float('nan'):.1f} us "
                  f"(100,000 segments)")
            for k in sorted(agg):
                print(f"  {k:28s} {agg[k]:14.4g}   per wave {agg[k] / waves:12.1f}")
            if agg.get("SQ_WAVE_CYCLES"):
                wc = agg["SQ_WAVE_CYCLES"]
                print(f"  wave lifetime split (quad-cycles): active {agg.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}, "
                      f"waiting {agg.get('SQ_WAIT_ANY', 0) / wc:.2f}, issue-stalled "
                      f"{agg.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}; VALU active {agg.get('SQ_ACTIVE_INST_VALU', 0) / wc:.2f}")

if __name__ == "__main__":
    main()
