# Round 6: counters of the LM's general path (ndata 30 / 62, config-2 QI, chunk size 1), before
# and after a change: kernel trace + stats, then one PMC pass per counter group
# (rocprofv3 does not split counters over passes). Usage: [LMSET='k=v;k=v'] bash scripts/gpu_lm_general_pmc.sh TAG
# (LMSET: the tuning sets of scripts/lm_pmc.py, one dfmi_lm launch each; default lm_general=0)
set -e
export TMPDIR=/tmp
TAG=${1:-lmgen}
O=gpurun_out/$TAG
mkdir -p $O
for ND in 30 62; do
  export ND SETTINGS="${LMSET:-lm_general=0}"
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/nd$ND/trace" -o lm -- python3 scripts/lm_pmc.py > $O/nd$ND.trace.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM --output-format csv -d "$PWD/$O/nd$ND/a" -o lm -- python3 scripts/lm_pmc.py > $O/nd$ND.a.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d "$PWD/$O/nd$ND/b" -o lm -- python3 scripts/lm_pmc.py > $O/nd$ND.b.log 2>&1
done
