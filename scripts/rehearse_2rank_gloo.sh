#!/bin/bash
# Rehearsal of bench.py's sharded path with 2 ranks sharing one GPU over gloo
# (the driver runs the real N-GPU bench over RCCL). Run from the repo root on the box.
set -o pipefail
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 WORLD_SIZE=2 DFMI_DIST_BACKEND=gloo
RANK=1 LOCAL_RANK=0 timeout -k 10 240 python -u bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/rh_r1.json 2> gpurun_out/rh_r1.err &
P1=$!
RANK=0 LOCAL_RANK=0 timeout -k 10 240 python -u bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/rh_r0.json 2> gpurun_out/rh_r0.err
R0=$?
wait $P1
R1=$?
echo "rc0=$R0 rc1=$R1"
cat gpurun_out/rh_r0.json; echo; wc -c gpurun_out/rh_r1.json
