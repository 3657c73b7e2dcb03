cd $GRAFT_REPO_ROOT
STEPS=tests,smoke,bench PYTEST_ARGS="--timeout 300" bash scripts/gpu_round.sh || exit $?
timeout -k 10 300 python scripts/probe_overlap.py > gpurun_out/probe_overlap.json 2> gpurun_out/probe_overlap.err; echo "probe rc=$?"; cat gpurun_out/probe_overlap.json; tail -3 gpurun_out/probe_overlap.err
