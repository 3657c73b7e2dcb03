# round 4, call u: the fused seed + demodulation kernel held to 168 VGPRs (3 waves per SIMD)
# against the uncapped build A (223 VGPRs, 2 waves), config 2 and the hard-seed record
set -o pipefail
mkdir -p gpurun_out
ROUNDS=7 timeout -k 10 300 python scripts/ab_libs.py > gpurun_out/r04u_ab.json 2> gpurun_out/r04u_ab.err || exit 1
cat gpurun_out/r04u_ab.json
PHI=1.3 PSI=0.4 ROUNDS=2 NSEG=100000 timeout -k 10 300 python scripts/ab_libs.py > gpurun_out/r04u_ab_hard.json 2> gpurun_out/r04u_ab_hard.err || exit 1
cat gpurun_out/r04u_ab_hard.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_numerics.py tests/test_gpu_parity.py -k "seed" -q --timeout 200 --timeout-method thread > gpurun_out/r04u_seed_tests.log 2>&1
tail -2 gpurun_out/r04u_seed_tests.log
