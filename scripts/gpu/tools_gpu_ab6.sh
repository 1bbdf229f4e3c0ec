#!/bin/bash
# full-region lane walk compiled in for K buckets > 40 only: A/B at K=16/50/64, then GPU tests + BASELINE suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/ab6.jsonl
: > $O
for k in 16 50 64 48; do
  timeout -k 10 120 python scripts/ab_lane.py 900000 $k 10 >> $O 2> gpurun_out/ab6.err || { echo AB_FAIL $k; tail -5 gpurun_out/ab6.err; exit 1; }
  tail -1 $O
done
bash scripts/gpu/tools_gpu_t7.sh
