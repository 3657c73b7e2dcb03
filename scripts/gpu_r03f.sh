#!/bin/bash
# round 3 session f: full GPU suite (flat worker gate, ladder, new tests), EKF A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
SETTINGS="ekf_v2=0;ekf_v2=1" timeout -k 10 300 python scripts/ekf_ab.py > gpurun_out/ekf_ab.json 2> gpurun_out/ekf_ab.err; rc=$?; echo "ekf_ab rc=$rc"; cat gpurun_out/ekf_ab.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/probe_pipeline.py > gpurun_out/probe_pipeline.json 2> gpurun_out/probe_pipeline.err; rc=$?; echo "pipeline rc=$rc"; cat gpurun_out/probe_pipeline.json
