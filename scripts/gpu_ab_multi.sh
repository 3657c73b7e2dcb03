#!/bin/bash
# A/B of several library builds in alternating processes on one box (scripts/step_time.py:
# config-2 ms/step + the demodulation alone + a checksum of the results): the in-tree build
# and every ab/libdfmi_*.so, ROUNDS times in turn. Stops at the first failure.
set -o pipefail
for i in $(seq 1 ${ROUNDS:-3}); do
  timeout -k 10 120 python scripts/step_time.py || exit 1
  for f in ab/libdfmi_*.so; do
    LIB=$PWD/$f timeout -k 10 120 python scripts/step_time.py || exit 1
  done
done
