# round 4, call t: the whole GPU suite, smoke() and the bench line after the EKF defaults moved
# (parallel in time up to 256 channels of >= 4096 samples)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread > gpurun_out/r04t_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r04t_pytest.log
grep -E "^FAILED|^ERROR" gpurun_out/r04t_pytest.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04t_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r04t_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r04t_bench.json 2> gpurun_out/r04t_bench.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/r04t_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_ms']); print(d['extra_configs']['config5']['one_channel'])"
exit $rc
