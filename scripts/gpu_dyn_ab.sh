# dynamic segment queues A/B (step + bit identity), then the per-wave finish spread, then GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 env SETTINGS="demod_dyn=0;demod_dyn=1" python scripts/tune_step.py > gpurun_out/tune_dyn.json 2>&1; rc=$?; cat gpurun_out/tune_dyn.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/demod_waves.py || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
