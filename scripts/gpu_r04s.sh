# round 4, call s: the convergence check folded into the pass kernel — PIT tests, then call r
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ekf_pit.py tests/test_gpu_parity.py -k "ekf or pit" -v -rP -x --timeout 200 --timeout-method thread > gpurun_out/r04s_pit.log 2>&1
rc=$?
tail -3 gpurun_out/r04s_pit.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/r04s_pit.log | head; exit $rc; fi
bash scripts/gpu_r04r.sh
