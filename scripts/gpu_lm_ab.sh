set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 env SETTINGS="lm_refill=0;lm_refill=1;lm_refill=1,lm_waves_per_simd=2" python scripts/tune_step.py > gpurun_out/tune_lm.json 2>&1; rc=$?; cat gpurun_out/tune_lm.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/bench20.json 2>&1; cat gpurun_out/bench20.json
