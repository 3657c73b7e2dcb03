# round 4, call b: seed-on-the-ladder + numerics tests (prints kept), hard-seed A/B against
# the round-3 build, the driver's bench command twice (window breakdown, new extra keys)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_numerics.py tests/test_gpu_full_scale.py tests/test_gpu_workers.py tests/test_gpu_multidevice.py tests/test_gpu_debug_build.py -v -rP --timeout 300 --timeout-method thread > gpurun_out/r04b_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r04b_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
PHI=1.3 PSI=0.4 ROUNDS=2 NSEG=100000 timeout -k 10 300 python scripts/ab_libs.py > gpurun_out/r04b_ab_hardseed.json 2> gpurun_out/r04b_ab_hardseed.err || exit 1
cat gpurun_out/r04b_ab_hardseed.json
for i in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04b_bench_driver$i.json 2> gpurun_out/r04b_bench_driver$i.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r04b_bench_driver$i.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['end_to_end_frac'], d['kernels_ms'], d['window_breakdown'])"
done
python -c "import json; d=json.load(open('gpurun_out/r04b_bench_driver1.json'))['extra_configs']; print(json.dumps(d['config2_end_to_end'])); print(json.dumps(d['config4_shard_1gpu']))"
exit $rc
