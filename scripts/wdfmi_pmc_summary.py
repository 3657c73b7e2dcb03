"""Summarise the witness fitters' SQ counters (scripts/gpu_r06.sh wdfmipmc: rocprofv3 --pmc over
scripts/bench_wdfmi.py --records 2048 --cpu 0 --reps 1) into profiles/rNN/wdfmi_pmc.txt.

Per dfmi_wdfmi_fit launch: waves, the dispatch's duration (Start/End timestamps of the counter
run, so with the counter overhead), wave-level VALU instructions, fp64 flops (FMA counted 2,
64 lanes per wave instruction: an upper bound, inactive lanes included) and their rate against
the fp64 vector peak, VGPRs. usage: python scripts/wdfmi_pmc_summary.py <counter_collection.csv>"""
import collections
import csv
import sys

METHOD = {"0": "wdfmi_nls", "1": "wdfmi_ortho", "2": "wdfmi_seq", "3": "hwdfmi"}
FP64_PEAK = 78.6e12  # fp64 vector FLOP/s, MI355X
BUFFERS = 2048 * 9


def main(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    info = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "wdfmi_fit_kernel<" not in k:
            continue
        d = int(r["Dispatch_Id"])
        agg[d][r["Counter_Name"]] += float(r["Counter_Value"])
        info[d] = (METHOD[k.split("wdfmi_fit_kernel<")[1].split(">")[0].split(",")[2].strip()],
                   (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9, r["VGPR_Count"])
    print("witness fitters: 2,048 records x 9 buffers, R = 4000 (the reference's 'cos' inputs), one "
          "dfmi_wdfmi_fit launch per line; SQ counters summed over the dispatch")
    print("method       disp  waves  dur_ms  VALU/wave  fp64 GFLOP  TFLOP/s  of_peak  MFLOP/buffer  vgpr")
    for d in sorted(agg):
        c, (m, dur, vg) = agg[d], info[d]
        w = c["SQ_WAVES"]
        fl = 64 * (2 * c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_ADD_F64"])
        print(f"{m:12s} {d:4d} {w:6.0f} {dur * 1e3:7.2f} {c['SQ_INSTS_VALU'] / w:10.3g} {fl / 1e9:11.1f} "
              f"{fl / dur / 1e12:8.2f} {fl / dur / FP64_PEAK:8.3f} {fl / BUFFERS / 1e6:13.2f}  {vg}")


if __name__ == "__main__":
    main(sys.argv[1])
