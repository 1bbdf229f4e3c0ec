#!/bin/bash
# K=50: the exact finish on the query stream (default) vs as a side-stream epilogue
# (KN_PIPE_EXACT=1), interleaved processes, 900K uniform, 200/50 and 20/5 steps.
set -e
mkdir -p gpurun_out
o=gpurun_out/ab_exact_k50.txt
: > $o
for rep in 1 2 3; do
  for ex in 0 1; do
    echo "== KN_PIPE_EXACT=$ex rep $rep" >> $o
    KN_PIPE_EXACT=$ex timeout -k 10 120 python bench.py --k 50 --steps 200 --warmup 50 --no-check >> $o 2>&1
    KN_PIPE_EXACT=$ex timeout -k 10 120 python bench.py --k 50 --steps 20 --warmup 5 --no-check >> $o 2>&1
  done
done
