# A/B of two library builds in one gpurun call, alternating processes on the same box:
# LIB_A (default in-tree) vs LIB_B, tune_step-style step time (config 2)
set -o pipefail
for i in 1 2 3; do
  timeout -k 10 120 python scripts/step_time.py || exit 1
  LIB=${LIB_B} timeout -k 10 120 python scripts/step_time.py || exit 1
done
