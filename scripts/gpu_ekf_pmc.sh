# PMC passes over the config-5 EKF (one channel): instructions and cycles per sample of
# ekf_rot_kernel<16>. One pass per counter group (rocprofv3 does not split counters),
# each under its own time limit; the script stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.." || exit 2
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/ekf_pmc_${TAG:-r04}
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
timeout -k 10 120 python3 scripts/ekf_pmc_target.py > "$OUT/plain.json" 2> "$OUT/plain.err" || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    --output-format csv -d "$OUT/p1" -o ekf -- python3 scripts/ekf_pmc_target.py > "$OUT/p1.json" 2> "$OUT/p1.err" || exit $?
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
    --output-format csv -d "$OUT/p2" -o ekf -- python3 scripts/ekf_pmc_target.py > "$OUT/p2.json" 2> "$OUT/p2.err" || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o ekf -- python3 scripts/ekf_pmc_target.py > "$OUT/trace.json" 2> "$OUT/trace.err" || exit $?
echo "ekf pmc ok"
