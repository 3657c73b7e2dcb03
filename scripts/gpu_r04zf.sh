# round 4, call zf (final: the rotation head): the whole GPU suite, smoke(), the driver's bench line, and the
# round's profiles of the driver's command (scripts/profile_round.sh, TAG=r04)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread > gpurun_out/r04zf_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r04zf_pytest.log
grep -E "^FAILED|^ERROR" gpurun_out/r04zf_pytest.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04zf_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r04zf_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r04zf_bench.json 2> gpurun_out/r04zf_bench.err || exit 1
python scripts/show_bench.py gpurun_out/r04zf_bench.json
TAG=r04zf bash scripts/profile_round.sh || exit 1
cat gpurun_out/prof_r04zf/window_check.json
exit $rc
