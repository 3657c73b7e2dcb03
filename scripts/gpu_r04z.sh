# round 4, call z: the channel-scaled block size — PIT tests, and the default path at 1..1024 channels
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ekf_pit.py tests/test_gpu_parity.py tests/test_gpu_full_scale.py -k "ekf or pit" -v -rP --timeout 300 --timeout-method thread > gpurun_out/r04z_pit.log 2>&1
rc=$?
tail -3 gpurun_out/r04z_pit.log
if [ $rc -ne 0 ]; then grep -E "Error|assert" gpurun_out/r04z_pit.log | head; exit $rc; fi
VARIANTS=0:256 CHANNELS=1,4,16,64,256,512,1024 REPS=2 timeout -k 10 600 python scripts/ekf_pit_ab.py > gpurun_out/r04z_ab.json 2> gpurun_out/r04z_ab.err || exit 1
tail -1 gpurun_out/r04z_ab.json | python -c "import json,sys; [print(v['channels'], v.get('kernel'), v['ms'], v.get('passes'), v.get('speedup_vs_seq')) for v in json.loads(sys.stdin.read())['variants']]"
