#!/bin/bash
# One parameterised GPU call (replaces round 4's one-off scripts/gpu_r04*.sh):
#   gpurun -- bash scripts/gpu_run.sh TAG STEP [STEP ...]
# Steps, run in order, each under its own time limit, outputs in gpurun_out/TAG_*:
#   tests              the whole GPU suite (pytest -m gpu)
#   tests=FILES_OR_K   pytest -m gpu on the given files (comma-separated), or -k EXPR if no
#                      entry ends in .py
#   smoke              __graft_entry__.smoke()
#   bench[=ARGS]       python bench.py ARGS (comma-separated) > TAG_bench.json
#   py=SCRIPT[,ARGS]   python -u SCRIPT ARGS > TAG_<script name>.jsonl
#   prof=SCRIPT[,ARGS] rocprofv3 --kernel-trace --stats of python SCRIPT ARGS -> TAG_prof/
#   pmc=COUNTERS=SCRIPT[,ARGS]  one rocprofv3 --pmc pass (COUNTERS space-free, '+'-joined)
#   round              scripts/profile_round.sh (the judged profiles of the driver's bench
#                      command: kernel trace + stats, PMC FETCH/WRITE, frac check) into
#                      gpurun_out/prof_TAG
# A step that fails stops the call: after a timeout (124/137), an abort (134) or a segfault
# (139) nothing else touches the GPU; a pytest failure (rc 1) still lets later steps run.
set -o pipefail
TAG=$1
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
rc_all=0
fatal() { case $1 in 124|134|137|139) return 0 ;; esac; [ "$1" -gt 128 ]; }
for step in "$@"; do
  name=${step%%=*}
  arg=""
  [ "$name" != "$step" ] && arg=${step#*=}
  echo "== $TAG $step ($(date +%T))"
  case $name in
    tests)
      sel=()
      if [ -n "$arg" ]; then
        IFS=',' read -ra parts <<< "$arg"
        if [[ "${parts[0]}" == *.py ]]; then sel=("${parts[@]}"); else sel=(-k "$arg"); fi
      else
        sel=(tests)
      fi
      timeout -k 10 1000 python -u -m pytest "${sel[@]}" -m gpu -v -rP --timeout 300 --timeout-method thread \
        > gpurun_out/${TAG}_pytest.log 2>&1
      rc=$?
      tail -3 gpurun_out/${TAG}_pytest.log
      grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_pytest.log | head -20
      ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
      rc=$?
      tail -2 gpurun_out/${TAG}_smoke.log
      ;;
    bench)
      IFS=',' read -ra bargs <<< "$arg"
      timeout -k 10 600 python bench.py "${bargs[@]}" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
      rc=$?
      [ $rc -eq 0 ] && python scripts/show_bench.py gpurun_out/${TAG}_bench.json
      [ $rc -ne 0 ] && tail -20 gpurun_out/${TAG}_bench.err
      ;;
    py)
      IFS=',' read -ra pargs <<< "$arg"
      out=gpurun_out/${TAG}_$(basename "${pargs[0]}" .py).jsonl
      timeout -k 10 600 python -u "${pargs[@]}" > "$out" 2> "${out%.jsonl}.err"
      rc=$?
      tail -c 3000 "$out"
      [ $rc -ne 0 ] && tail -20 "${out%.jsonl}.err"
      ;;
    prof)
      IFS=',' read -ra pargs <<< "$arg"
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 "${pargs[@]}" \
        > gpurun_out/${TAG}_prof.log 2>&1
      rc=$?
      tail -5 gpurun_out/${TAG}_prof.log
      ;;
    pmc)
      counters=${arg%%=*}
      rest=${arg#*=}
      IFS=',' read -ra pargs <<< "$rest"
      timeout -s KILL 120 rocprofv3 --pmc ${counters//+/ } -d gpurun_out/${TAG}_pmc_${counters//+/_} -o run \
        -- python3 "${pargs[@]}" > gpurun_out/${TAG}_pmc.log 2>&1
      rc=$?
      tail -3 gpurun_out/${TAG}_pmc.log
      ;;
    round)
      TAG=$TAG timeout -k 10 1500 bash scripts/profile_round.sh > gpurun_out/${TAG}_round.log 2>&1
      rc=$?
      tail -3 gpurun_out/${TAG}_round.log
      ;;
    *)
      echo "unknown step $step"
      rc=2
      ;;
  esac
  echo "== $TAG $step rc=$rc ($(date +%T))"
  [ $rc -ne 0 ] && rc_all=$rc
  if fatal $rc; then exit $rc; fi
  if [ $rc -ne 0 ] && [ "$name" != "tests" ]; then exit $rc; fi
done
exit $rc_all
