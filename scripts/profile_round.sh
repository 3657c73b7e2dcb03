#!/bin/bash
# rocprofv3 passes for the judged profiles (run on the GPU box via gpurun):
#  1) --kernel-trace --stats over the default bench command (no CPU baseline)
#  2) PMC pass: FETCH_SIZE       over the demod-only bench
#  3) PMC pass: WRITE_SIZE       over the demod-only bench
#  4) profiles/pmc_demod.json from 2) + 3) (scripts/pmc_summary.py)
# Each step has its own time limit; the script stops at the first failure.
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/prof_${TAG:-r01}
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- \
    python3 bench.py --no-cpu-baseline > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o demod -- \
    python3 bench.py --demod-only --steps 10 --warmup 2 > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err" || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o demod -- \
    python3 bench.py --demod-only --steps 10 --warmup 2 > "$OUT/pmc_write.json" 2> "$OUT/pmc_write.err" || exit $?
KERN=$(python3 -c "import json; print(json.load(open('$OUT/pmc_fetch.json'))['roofline']['kernel'].split('<')[0])") || exit 3
python3 scripts/pmc_summary.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$KERN" 3216800000 \
    "bench.py --demod-only --steps 10 --warmup 2 (100000 segments, R=4000, ndata=10)" > "$OUT/pmc_summary.json" || exit $?
cp profiles/pmc_demod.json "$OUT/" 
echo "profile ok"
