# round 4, call i: EKF parallel in time with the sequential head — tests, A/B, kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ekf_pit.py -v -rP --timeout 200 --timeout-method thread > gpurun_out/r04i_pit.log 2>&1
rc=$?
tail -3 gpurun_out/r04i_pit.log
grep "passes" gpurun_out/r04i_pit.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VARIANTS=0:512,0:0,25:512,25:256,49:1024,16:512 CHANNELS=1,4 timeout -k 10 200 python scripts/ekf_pit_ab.py > gpurun_out/r04i_ab.json 2> gpurun_out/r04i_ab.err || exit 1
tail -1 gpurun_out/r04i_ab.json | python -c "import json,sys; [print(v) for v in json.loads(sys.stdin.read())['variants']]"
VARIANTS=0:512 REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04i_prof -o run -- python scripts/ekf_pit_ab.py > gpurun_out/r04i_prof.log 2>&1 || exit 1
f=$(find gpurun_out/r04i_prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -14
exit $rc
