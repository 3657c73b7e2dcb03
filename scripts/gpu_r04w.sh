# round 4, call w: EKF parallel in time — block size and head length around the defaults
set -o pipefail
mkdir -p gpurun_out
VARIANTS=0:256,16:256,20:256,32:256,0:192,0:384 CHANNELS=1,16 REPS=5 timeout -k 10 400 python scripts/ekf_pit_ab.py > gpurun_out/r04w_ab.json 2> gpurun_out/r04w_ab.err || exit 1
tail -1 gpurun_out/r04w_ab.json | python -c "import json,sys; [print(v) for v in json.loads(sys.stdin.read())['variants']]"
