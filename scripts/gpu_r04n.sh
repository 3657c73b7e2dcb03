# round 4, call n: the whole GPU suite, smoke(), the default bench line (the driver's commands)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread > gpurun_out/r04n_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r04n_pytest.log
grep -E "FAILED|ERROR" gpurun_out/r04n_pytest.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04n_smoke.log 2>&1 || exit 1
tail -2 gpurun_out/r04n_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r04n_bench.json 2> gpurun_out/r04n_bench.err || exit 1
tail -1 gpurun_out/r04n_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac']); print(json.dumps(d['extra']['config5'] if 'extra' in d else d.get('config5'))[:1500])"
exit $rc
