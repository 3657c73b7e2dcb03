# LM two-phase A/B (step time, bit identity) + LM-only probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 env SETTINGS="lm_phase=0;lm_phase=1;lm_phase=1,lm_pa=2;lm_phase=1,lm_pa=4;lm_phase=1,lm_pa_w2=0" python scripts/tune_step.py > gpurun_out/tune_lm_phase.json 2>&1; rc=$?; cat gpurun_out/tune_lm_phase.json; [ $rc -eq 0 ] || exit $rc
