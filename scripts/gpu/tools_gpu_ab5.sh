#!/bin/bash
# lane walk over the whole staged block vs the lane's own +-H box vs the union stream, then GPU tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/ab5.jsonl
: > $O
for k in 16 50 32 8 64; do
  timeout -k 10 120 python scripts/ab_lane.py 900000 $k 10 >> $O 2> gpurun_out/ab5.err || { echo AB_FAIL $k; tail -5 gpurun_out/ab5.err; exit 1; }
  tail -1 $O
done
timeout -k 10 120 python scripts/ab_lane.py 300000 16 10 >> $O 2> gpurun_out/ab5.err || { echo AB_FAIL 300k; tail -5 gpurun_out/ab5.err; exit 1; }
timeout -k 10 200 python scripts/ab_lane.py 900000 16 3 clustered >> $O 2> gpurun_out/ab5.err || { echo AB_FAIL cl; tail -5 gpurun_out/ab5.err; exit 1; }
tail -2 $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab5_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/ab5_tests.log; exit 1; }
tail -1 gpurun_out/ab5_tests.log
