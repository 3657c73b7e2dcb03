# round 4, call ze: the moments tree with its plan levels and chain staged in LDS — the moments /
# EKF GPU tests, one-channel timing, kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ekf_pit.py tests/test_gpu_parity.py tests/test_gpu_numerics.py -m gpu -k "ekf or pit or moment" -v -rP --timeout 300 --timeout-method thread > gpurun_out/r04ze_pit.log 2>&1
rc=$?
tail -3 gpurun_out/r04ze_pit.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|Error|assert" gpurun_out/r04ze_pit.log | head; exit $rc; fi
VARIANTS=0:256 CHANNELS=1 REPS=7 timeout -k 10 300 python scripts/ekf_pit_ab.py > gpurun_out/r04ze_ab.json 2> gpurun_out/r04ze_ab.err || exit 1
tail -1 gpurun_out/r04ze_ab.json | python -c "import json,sys; [print(v['channels'], v.get('kernel'), v['ms'], v.get('passes')) for v in json.loads(sys.stdin.read())['variants']]"
VARIANTS=0:256 REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04ze_prof -o run -- python scripts/ekf_pit_ab.py > gpurun_out/r04ze_prof.log 2>&1 || exit 1
