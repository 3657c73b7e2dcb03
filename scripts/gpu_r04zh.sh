# round 4, call zh: the whole GPU suite, smoke() and the bench line at the final HEAD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread > gpurun_out/r04zh_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r04zh_pytest.log
grep -E "^FAILED|^ERROR" gpurun_out/r04zh_pytest.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04zh_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r04zh_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r04zh_bench.json 2> gpurun_out/r04zh_bench.err || exit 1
python scripts/show_bench.py gpurun_out/r04zh_bench.json
exit $rc
