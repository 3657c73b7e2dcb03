# round 4, call zg: what the launches after convergence cost (pass budget 6 / 8 / 12, config 5 converges in 5)
set -o pipefail
mkdir -p gpurun_out
for p in 6 8 12; do
  PASSES=$p VARIANTS=0:256 CHANNELS=1 REPS=9 timeout -k 10 200 python scripts/ekf_pit_ab.py > gpurun_out/r04zg_p$p.json 2> gpurun_out/r04zg_p$p.err || exit 1
  tail -1 gpurun_out/r04zg_p$p.json | python -c "import json,sys; v=json.loads(sys.stdin.read())['variants'][1]; print($p, v['ms'], v['passes'])"
done
