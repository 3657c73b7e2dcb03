# round 4, call y: EKF parallel in time — larger blocks for many channels
set -o pipefail
mkdir -p gpurun_out
VARIANTS=64:256,128:256,256:256 CHANNELS=16 REPS=3 timeout -k 10 300 python scripts/ekf_pit_ab.py > gpurun_out/r04y_16.json 2> gpurun_out/r04y_16.err || exit 1
VARIANTS=256:256,512:256,1024:256 CHANNELS=64 REPS=3 timeout -k 10 300 python scripts/ekf_pit_ab.py > gpurun_out/r04y_64.json 2> gpurun_out/r04y_64.err || exit 1
VARIANTS=512:256,1024:256,2048:256,4096:256 CHANNELS=256 REPS=2 timeout -k 10 400 python scripts/ekf_pit_ab.py > gpurun_out/r04y_256.json 2> gpurun_out/r04y_256.err || exit 1
for f in 16 64 256; do tail -1 gpurun_out/r04y_$f.json | python -c "import json,sys; [print(v['channels'], v.get('kernel'), v['ms'], v.get('passes')) for v in json.loads(sys.stdin.read())['variants']]"; done
