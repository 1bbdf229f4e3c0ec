#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python bench.py --loopback 8 --n 12500000 --k 16 --steps 3 --warmup 1 > gpurun_out/loop100m.json 2> gpurun_out/loop100m.err || { echo LOOP_FAIL; tail gpurun_out/loop100m.err; exit 1; }
cat gpurun_out/loop100m.json
for k in 50 32 16; do
  timeout -k 10 300 python scripts/sweep_tiles.py 900000 $k > gpurun_out/sweep_k$k.log 2>&1 || { echo SWEEP_FAIL $k; tail gpurun_out/sweep_k$k.log; exit 1; }
  grep BEST gpurun_out/sweep_k$k.log
done
