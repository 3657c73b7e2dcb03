# round 4, call e: the hard-seed step split (fused vs LM, seed fit time from the probe),
# and the EKF prefetch-distance A/B (1 vs 2 groups ahead), alternating processes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python scripts/probe_seed_hard.py > gpurun_out/r04e_probe_seed.json 2> gpurun_out/r04e_probe_seed.err || exit 1
cat gpurun_out/r04e_probe_seed.json
for i in 1 2; do
  LIBS="pf1=$PWD/deepfmkit_amd/libdfmi.so;pf2=$PWD/ab/libdfmi_pf2.so" timeout -k 10 200 python scripts/ekf_ab.py > gpurun_out/r04e_ekf_pf_ab$i.json 2> gpurun_out/r04e_ekf_pf_ab$i.err || exit 1
  cat gpurun_out/r04e_ekf_pf_ab$i.json
done
