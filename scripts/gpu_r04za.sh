# round 4, call za: the EKF / PIT GPU tests under -m gpu (the channel-scaled block size), and
# whether torch sees the GPU after the library initialised HIP first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python scripts/probe_init_order.py > gpurun_out/r04za_init_order.json 2> gpurun_out/r04za_init_order.err; cat gpurun_out/r04za_init_order.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_ekf_pit.py tests/test_gpu_parity.py tests/test_gpu_full_scale.py -m gpu -k "ekf or pit" -v -rP --timeout 300 --timeout-method thread > gpurun_out/r04za_pit.log 2>&1
rc=$?
tail -3 gpurun_out/r04za_pit.log
grep -E "^FAILED|^ERROR" gpurun_out/r04za_pit.log | head
exit $rc
