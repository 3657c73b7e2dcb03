# round 4, call o: the large-argument J0/J1 out of line (lm_chunks_kernel back to 248 VGPRs,
# 2 waves per SIMD) against the inlined build A, config 2 and the hard-seed record
set -o pipefail
mkdir -p gpurun_out
ROUNDS=5 timeout -k 10 300 python scripts/ab_libs.py > gpurun_out/r04o_ab.json 2> gpurun_out/r04o_ab.err || exit 1
cat gpurun_out/r04o_ab.json
PHI=1.3 PSI=0.4 ROUNDS=2 NSEG=100000 timeout -k 10 300 python scripts/ab_libs.py > gpurun_out/r04o_ab_hard.json 2> gpurun_out/r04o_ab_hard.err || exit 1
cat gpurun_out/r04o_ab_hard.json
