# PMC passes over scripts/lm_pmc.py (each counter set its own run)
export TMPDIR=/tmp
mkdir -p gpurun_out/lm_pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$PWD/gpurun_out/lm_pmc/a" -o lm -- python3 scripts/lm_pmc.py > gpurun_out/lm_pmc/a.log 2>&1 || { tail -5 gpurun_out/lm_pmc/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM --output-format csv -d "$PWD/gpurun_out/lm_pmc/b" -o lm -- python3 scripts/lm_pmc.py > gpurun_out/lm_pmc/b.log 2>&1 || { tail -5 gpurun_out/lm_pmc/b.log; exit 1; }
find gpurun_out/lm_pmc -name "*counter_collection*" | head
