# round 4, call d: the post-sync slowdown probe; seed timings with full evaluations on the
# ladder; the general (flat) path A/B against round 3 (lm_general=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python scripts/probe_sync.py > gpurun_out/r04d_probe_sync.json 2> gpurun_out/r04d_probe_sync.err || exit 1
cat gpurun_out/r04d_probe_sync.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_numerics.py -k "seed or ladder" -v -rP --timeout 200 --timeout-method thread > gpurun_out/r04d_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/r04d_pytest.log
grep "noise_only=" gpurun_out/r04d_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TUNE=lm_general=1 ROUNDS=3 timeout -k 10 300 python scripts/ab_libs.py > gpurun_out/r04d_ab_general.json 2> gpurun_out/r04d_ab_general.err || exit 1
cat gpurun_out/r04d_ab_general.json
exit $rc
