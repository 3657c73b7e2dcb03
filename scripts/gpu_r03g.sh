#!/bin/bash
# round 3 session g: worker tests (resolution gate), bench with the extra configs
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_workers.py tests/test_gpu_parity.py -q -p no:cacheprovider --timeout 120 > gpurun_out/pytest_g.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_g.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_g.json 2> gpurun_out/bench_g.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_g.json; tail -3 gpurun_out/bench_g.err
