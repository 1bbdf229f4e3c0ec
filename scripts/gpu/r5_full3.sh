#!/bin/bash
# distributed diag (every capture mode) + full GPU suite + smoke + benches (engine, dist)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5full3
mkdir -p $O
MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 WORLD_SIZE=1 timeout -k 10 400 python -u scripts/diag_dist_pipe.py 30 200000 > $O/diag.log 2>&1 || { echo DIAG_FAIL; tail -30 $O/diag.log; exit 1; }
grep -E "ALL OK|FAIL" $O/diag.log | tail -3
OUT_DIR=r5full3 bash scripts/gpu/r5_full.sh
