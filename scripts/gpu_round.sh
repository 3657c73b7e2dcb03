#!/bin/bash
# One gpurun call: GPU tests, smoke, bench, rocprofv3 kernel stats.
# Stops at the first step that crashes/aborts/times out (exit codes other than
# 0 = pass and 1 = test failures).
cd "$(dirname "$0")/.." || exit 2
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
STEPS=${STEPS:-tests,smoke,bench,prof}
if [[ $STEPS == *tests* ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log
  ok $rc || exit $rc
fi
if [[ $STEPS == *smoke* ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
  ok $rc || exit $rc
fi
if [[ $STEPS == *bench* ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
  [ $rc -eq 0 ] || exit $rc
fi
if [[ $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof" -o run --output-format csv -- \
      python3 bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.err
  find gpurun_out/prof -name '*stats*' | head
fi
exit 0
