#!/bin/bash
# round 3 session i: EKF one-channel kernel (lane-split sincos, DPP destinations)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -k "ekf or EKF" -q -p no:cacheprovider --timeout 120 > gpurun_out/pytest_i.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_i.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
SETTINGS="ekf_row=1;ekf_row=0" timeout -k 10 300 python scripts/ekf_ab.py > gpurun_out/ekf_ab_i.json 2> gpurun_out/ekf_ab_i.err; rc=$?; echo "ekf_ab rc=$rc"; cat gpurun_out/ekf_ab_i.json
