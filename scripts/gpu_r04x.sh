# round 4, call x: EKF parallel in time — block size for many channels
set -o pipefail
mkdir -p gpurun_out
VARIANTS=0:256,32:256,64:256,128:256 CHANNELS=4,64,128 REPS=3 timeout -k 10 600 python scripts/ekf_pit_ab.py > gpurun_out/r04x_ab.json 2> gpurun_out/r04x_ab.err || exit 1
tail -1 gpurun_out/r04x_ab.json | python -c "import json,sys; [print(v) for v in json.loads(sys.stdin.read())['variants']]"
