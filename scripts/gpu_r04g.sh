# round 4, call g: large-argument Bessel (runaway descents) — the whole GPU suite, the
# hard-seed probe, the hard-record step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread > gpurun_out/r04g_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r04g_pytest.log
grep "noise_only=\|per-trial\|vs the oracle =" gpurun_out/r04g_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python scripts/probe_seed_hard.py > gpurun_out/r04g_probe_seed.json 2> gpurun_out/r04g_probe_seed.err || exit 1
cat gpurun_out/r04g_probe_seed.json
PHI=1.3 PSI=0.4 ROUNDS=2 NSEG=100000 timeout -k 10 300 python scripts/ab_libs.py > gpurun_out/r04g_ab_hardseed.json 2> gpurun_out/r04g_ab_hardseed.err || exit 1
cat gpurun_out/r04g_ab_hardseed.json
exit $rc
