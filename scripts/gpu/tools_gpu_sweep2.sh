#!/bin/bash
# grid density / halo sweep of the lane-walk default at K=50 and K=32 (900K uniform)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python scripts/sweep_tiles.py 900000 50 2.2,2.9,3.4,4.0,5.0 4x4x4,4x4x2 0,2,3 > gpurun_out/sweep2_k50.log 2>&1 || { echo SWEEP_FAIL 50; tail gpurun_out/sweep2_k50.log; exit 1; }
grep BEST gpurun_out/sweep2_k50.log
timeout -k 10 300 python scripts/sweep_tiles.py 900000 32 2.9,3.4,4.0,5.0 4x4x4,4x4x2 0,2,3 > gpurun_out/sweep2_k32.log 2>&1 || { echo SWEEP_FAIL 32; tail gpurun_out/sweep2_k32.log; exit 1; }
grep BEST gpurun_out/sweep2_k32.log
