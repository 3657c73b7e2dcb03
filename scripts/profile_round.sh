#!/bin/bash
# rocprofv3 passes for the judged profiles (run on the GPU box via gpurun):
#  1) --kernel-trace --marker-trace --stats over the driver's exact bench command
#     (bench.py --gpus 1 --steps 20 --warmup 5); window_check.json accounts its timed window
#     (the roctx range bench.py puts around it) from that trace
#  2) PMC pass: FETCH_SIZE over a short bench run (the step's fused kernel)
#  3) PMC pass: WRITE_SIZE over the same
#  4) profiles/pmc_demod.json from 2) + 3) (scripts/pmc_summary.py), for the step's
#     own dominant kernel (demod_seed_bins_kernel)
#  5) frac_check.json: the line's roofline fraction recomputed from 1)'s kernel trace
# Each step has its own time limit; the script stops at the first failure.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof_${TAG:-r04}
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || exit $?
python3 scripts/window_check.py "$OUT/trace" 20 > "$OUT/window_check.json" || true
PMC_CMD="bench.py --no-cpu-baseline --no-extra --steps 5 --warmup 1"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o step -- \
    python3 $PMC_CMD > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err" || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o step -- \
    python3 $PMC_CMD > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err" || exit $?
KERN=$(python3 -c "import json; print(json.load(open('$OUT/pmc_fetch.json'))['roofline']['kernel'].split('<')[0])") || exit 3
python3 scripts/pmc_summary.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$KERN" 3216800000 \
    "$PMC_CMD (100000 segments, R=4000, ndata=10)" > "$OUT/pmc_summary.json" || exit $?
cp profiles/pmc_demod.json "$OUT/"
python3 scripts/frac_check.py "$OUT/bench_trace.json" "$OUT/trace/bench_kernel_trace.csv" > "$OUT/frac_check.json" || exit $?
echo "profile ok"
