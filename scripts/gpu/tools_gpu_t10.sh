#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dist2 -o run -- python3 $R/bench.py --dist --no-check --steps 20 --warmup 3 > $R/gpurun_out/prof_dist2.log 2>&1 || { echo PROF_FAIL; tail $R/gpurun_out/prof_dist2.log; exit 1; }
echo PROF_OK
