# round 4, call m: PMC passes over the EKF parallel-in-time kernels (one channel, config 5)
set -o pipefail
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r04m_pmc
mkdir -p "$OUT"
export VARIANTS=0:256 CHANNELS=1 REPS=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS \
    --output-format csv -d "$OUT/p1" -o pit -- python3 scripts/ekf_pit_ab.py > "$OUT/p1.json" 2> "$OUT/p1.err" || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM \
    --output-format csv -d "$OUT/p2" -o pit -- python3 scripts/ekf_pit_ab.py > "$OUT/p2.json" 2> "$OUT/p2.err" || exit $?
echo "pit pmc ok"
