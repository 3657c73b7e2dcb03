# Round-6 GPU session helper: pytest selections + profiles, each step under its own limit,
# stopping at the first failure. Usage: bash scripts/gpu_r06.sh TAG STEP...
#   steps: full (many-harmonic / short-segment full-scale parity), quick (quickstart fixtures),
#          ekf (EKF parallel-in-time tests + stress), lmpmc (LM general-path counters), suite (all -m gpu),
#          bench (python bench.py), wdfmi (witness fitters bench + kernel stats)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
PYT="python -u -m pytest -x -v -s --timeout 600 --timeout-method thread"
for step in "$@"; do
  case $step in
    full) timeout -k 10 900 $PYT tests/test_gpu_full_scale.py -k many_harmonics > $O/full.log 2>&1 || exit 11 ;;
    quick) timeout -k 10 300 $PYT tests/test_gpu_quickstart.py > $O/quick.log 2>&1 || exit 12 ;;
    ekf) timeout -k 10 600 $PYT tests/test_gpu_ekf_pit.py tests/test_gpu_ekf_pit_stress.py > $O/ekf.log 2>&1 || exit 13 ;;
    lmpmc) timeout -k 10 600 bash scripts/gpu_lm_general_pmc.sh $TAG/lmpmc > $O/lmpmc.log 2>&1 || exit 14 ;;
    suite) timeout -k 10 1500 $PYT -m gpu tests > $O/suite.log 2>&1 || exit 15 ;;
    bench) timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 16 ;;
    wdfmi) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/wdfmi_prof" -o wd -- python3 scripts/bench_wdfmi.py > $O/wdfmi.jsonl 2> $O/wdfmi.err || exit 17 ;;
    sweep) timeout -k 10 300 python -u scripts/probe_ndata_sweep.py 100000 > $O/sweep.jsonl 2> $O/sweep.err || exit 18
           timeout -k 10 300 python -u scripts/probe_ndata_sweep.py 100000 lm_wide=0 > $O/sweep_literal.jsonl 2>> $O/sweep.err || exit 18 ;;
    sweepnolds) timeout -k 10 300 python -u scripts/probe_ndata_sweep.py 100000 lm_wide_lds=0 > $O/sweep_nolds.jsonl 2>> $O/sweep.err || exit 21 ;;
    sweepx) for spec in $SWEEPS; do  # SWEEPS="name:key=v+key=v ..."
              timeout -k 10 300 python -u scripts/probe_ndata_sweep.py 100000 "${spec#*:}" > $O/sweep_${spec%%:*}.jsonl 2>> $O/sweep.err || exit 22
            done ;;
    ekfho) timeout -k 10 300 python -u scripts/probe_ekf_handover.py > $O/ekf_handover.jsonl 2> $O/ekf_handover.err || exit 23
           MODES=2 REPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/ekfho_prof" -o ho -- python3 scripts/probe_ekf_handover.py > $O/ekf_handover_prof.jsonl 2>> $O/ekf_handover.err || exit 23 ;;
    wdfmipmc) timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 --output-format csv -d "$PWD/$O/wdfmi_pmc" -o wd -- python3 scripts/bench_wdfmi.py --records 2048 --cpu 0 --reps 1 > $O/wdfmi_pmc.jsonl 2> $O/wdfmi_pmc.err || exit 24 ;;
    lmvec) timeout -k 10 600 $PYT tests/test_gpu_lm_stress.py tests/test_gpu_parity.py tests/test_gpu_numerics.py > $O/lmvec.log 2>&1 || exit 19 ;;
    pitmoves) timeout -k 10 300 python -u scripts/probe_pit_moves.py > $O/pit_moves.jsonl 2> $O/pit_moves.err || exit 20 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step ok"
done
