# round 4, call c: general-path split evaluator (seed) tests + timings, hard-seed A/B,
# facade profile, EKF PMC passes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_numerics.py tests/test_gpu_parity.py tests/test_gpu_edge_records.py -v -rP --timeout 300 --timeout-method thread > gpurun_out/r04c_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r04c_pytest.log
grep "noise_only=" gpurun_out/r04c_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
PHI=1.3 PSI=0.4 ROUNDS=2 NSEG=100000 timeout -k 10 300 python scripts/ab_libs.py > gpurun_out/r04c_ab_hardseed.json 2> gpurun_out/r04c_ab_hardseed.err || exit 1
cat gpurun_out/r04c_ab_hardseed.json
timeout -k 10 300 python scripts/profile_facade.py > gpurun_out/r04c_facade.json 2> gpurun_out/r04c_facade.err || exit 1
cat gpurun_out/r04c_facade.json
TAG=r04c timeout -k 10 600 bash scripts/gpu_ekf_pmc.sh || exit 1
exit $rc
