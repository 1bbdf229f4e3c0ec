#!/bin/bash
# LDS capacity / occupancy sweep of the default (lane-walk) query kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/cap.jsonl
: > $O
timeout -k 10 120 python scripts/sweep_cap.py 900000 16 2048,1920,1856,1792,1728 >> $O 2> gpurun_out/cap.err || { echo CAP_FAIL; tail gpurun_out/cap.err; exit 1; }
timeout -k 10 200 python scripts/sweep_cap.py 10000000 16 2048,1856,1792 >> $O 2> gpurun_out/cap.err || { echo CAP_FAIL; tail gpurun_out/cap.err; exit 1; }
timeout -k 10 200 python scripts/sweep_cap.py 10000000 32 2048,1856,1792 >> $O 2> gpurun_out/cap.err || { echo CAP_FAIL; tail gpurun_out/cap.err; exit 1; }
cat $O
