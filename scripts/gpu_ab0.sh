#!/bin/bash
# in-process A/B of library builds under ab/ (scripts/ab_libs.py), phi = 0 only
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=""; for f in ab/libdfmi_*.so; do n=$(basename $f .so); L="$L;${n#libdfmi_}=$PWD/$f"; done; L=${L#;}
LIBS="$L" SEQALL=${SEQALL:-0} timeout -k 10 300 python scripts/ab_libs.py > gpurun_out/ab0.json 2> gpurun_out/ab0.err; rc=$?; echo "ab phi0 rc=$rc"; cat gpurun_out/ab0.json; tail -3 gpurun_out/ab0.err
