#!/bin/bash
# EKF A/B of library builds under ab/ (scripts/ekf_ab.py LIBS=...)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=""; for f in ab/libdfmi_*.so; do n=$(basename $f .so); L="$L;${n#libdfmi_}=$PWD/$f"; done; L=${L#;}
LIBS="$L" timeout -k 10 300 python scripts/ekf_ab.py > gpurun_out/ekf_ab_libs.json 2> gpurun_out/ekf_ab_libs.err; rc=$?; echo "ekf_ab rc=$rc"; cat gpurun_out/ekf_ab_libs.json; tail -3 gpurun_out/ekf_ab_libs.err
