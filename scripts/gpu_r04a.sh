# round 4, call a: GPU suite (incl. the full-scale parity against the numpy oracle), the
# psi-rotation A/B against the round-3 build (ab/libdfmi_A.so), and the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04a_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r04a_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
ROUNDS=5 timeout -k 10 300 python scripts/ab_libs.py > gpurun_out/r04a_ab.json 2> gpurun_out/r04a_ab.err || exit 1
cat gpurun_out/r04a_ab.json
timeout -k 10 400 python bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/r04a_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels_ms'])"
exit $rc
