# round 4, call f: lm_park bit identity + A/B (config 2, hard record), hard-seed probe,
# EKF prefetch-distance A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_numerics.py -k "park or seed or ladder" -v -rP --timeout 200 --timeout-method thread > gpurun_out/r04f_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/r04f_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
BITS=1 SETTINGS="lm_park=0;lm_park=2;lm_park=4;lm_park=8" timeout -k 10 300 python scripts/tune_step.py > gpurun_out/r04f_park_c2.json 2> gpurun_out/r04f_park_c2.err || exit 1
cat gpurun_out/r04f_park_c2.json
PHI=1.3 PSI=0.4 BITS=1 SETTINGS="lm_park=0;lm_park=4;lm_park=8" timeout -k 10 300 python scripts/tune_step.py > gpurun_out/r04f_park_hard.json 2> gpurun_out/r04f_park_hard.err || exit 1
cat gpurun_out/r04f_park_hard.json
timeout -k 10 200 python scripts/probe_seed_hard.py > gpurun_out/r04f_probe_seed.json 2> gpurun_out/r04f_probe_seed.err || exit 1
cat gpurun_out/r04f_probe_seed.json
LIBS="pf1=$PWD/deepfmkit_amd/libdfmi.so;pf2=$PWD/ab/libdfmi_pf2.so" timeout -k 10 200 python scripts/ekf_ab.py > gpurun_out/r04f_ekf_pf_ab.json 2> gpurun_out/r04f_ekf_pf_ab.err || exit 1
cat gpurun_out/r04f_ekf_pf_ab.json
