# round 4, call r: where the EKF parallel in time pays (channel counts, short records), and the
# driver's command under a kernel + marker trace (the timed window accounted by window_check.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_ekf_pit.py tests/test_gpu_full_scale.py -k "ekf or pit" -v -rP --timeout 300 --timeout-method thread > gpurun_out/r04r_pit.log 2>&1
rc=$?
tail -3 gpurun_out/r04r_pit.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/r04r_pit.log | head; exit $rc; fi
for sec in 0.01 0.02 0.05 0.1; do
  R_=400 SECONDS_=$sec PITMIN=1024 VARIANTS=0:256 CHANNELS=1,8 REPS=5 timeout -k 10 200 python scripts/ekf_pit_ab.py > gpurun_out/r04r_short_$sec.json 2> gpurun_out/r04r_short_$sec.err || exit 1
  tail -1 gpurun_out/r04r_short_$sec.json
done
OUT=gpurun_out/prof_r04r
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $OUT/trace -o bench -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_trace.json 2> $OUT/trace.err || exit 1
ls $OUT/trace
python3 scripts/window_check.py $OUT/trace 20 > $OUT/window_check.json; cat $OUT/window_check.json
