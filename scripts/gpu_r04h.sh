# round 4, call h: the EKF parallel in time — its tests, the EKF parity tests, the block-size A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ekf_pit.py -v -rP -x --timeout 200 --timeout-method thread > gpurun_out/r04h_pit.log 2>&1
rc=$?
tail -5 gpurun_out/r04h_pit.log
grep "passes" gpurun_out/r04h_pit.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python scripts/ekf_pit_ab.py > gpurun_out/r04h_ab.json 2> gpurun_out/r04h_ab.err || exit 1
cat gpurun_out/r04h_ab.json
exit $rc
