# round 4, call p: EKF + fold fused per pass (ekf_pit_pass_kernel) — PIT tests, A/B fused vs not, kernel trace;
# then the out-of-line large-argument Bessel A/B (call o)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ekf_pit.py -v -rP -x --timeout 200 --timeout-method thread > gpurun_out/r04p_pit.log 2>&1
rc=$?
tail -3 gpurun_out/r04p_pit.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/r04p_pit.log | head; exit $rc; fi
VARIANTS=0:256 CHANNELS=1,8 timeout -k 10 200 python scripts/ekf_pit_ab.py > gpurun_out/r04p_ab.json 2> gpurun_out/r04p_ab.err || exit 1
FUSED=0 VARIANTS=0:256 CHANNELS=1,8 timeout -k 10 200 python scripts/ekf_pit_ab.py > gpurun_out/r04p_ab_unfused.json 2> gpurun_out/r04p_ab_unfused.err || exit 1
tail -1 gpurun_out/r04p_ab.json; tail -1 gpurun_out/r04p_ab_unfused.json
VARIANTS=0:256 REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04p_prof -o run -- python scripts/ekf_pit_ab.py > gpurun_out/r04p_prof.log 2>&1 || exit 1
bash scripts/gpu_r04o.sh
