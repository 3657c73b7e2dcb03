# round 4, call zb: torch after a library-first host-memory call, with _lib.load importing torch first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python scripts/probe_init_order.py > gpurun_out/r04zb_init_order.json 2> gpurun_out/r04zb_init_order.err; cat gpurun_out/r04zb_init_order.json; tail -3 gpurun_out/r04zb_init_order.err
