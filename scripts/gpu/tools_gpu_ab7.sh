#!/bin/bash
# two-phase vs own-box lane walk at the 3-ring-halo plans (K=48/50/64)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/ab7.jsonl
: > $O
for k in 50 64 48; do
  timeout -k 10 120 python scripts/ab_lane.py 900000 $k 10 >> $O 2> gpurun_out/ab7.err || { echo AB_FAIL $k; tail -5 gpurun_out/ab7.err; exit 1; }
done
timeout -k 10 200 python scripts/ab_lane.py 3000000 50 6 >> $O 2> gpurun_out/ab7.err || { echo AB_FAIL 3m; tail -5 gpurun_out/ab7.err; exit 1; }
cat $O
