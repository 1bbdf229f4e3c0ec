#!/bin/bash
# Top-K margin 1 (_C_m1) vs 2 (_C) for K <= 32 with the exact finish as a side-stream epilogue
# (KN_PIPE_EXACT=1), and the default placement for reference; 900K uniform, in-process interleaved.
set -e
mkdir -p gpurun_out
export PYTHONPATH=$PWD
o=gpurun_out/ab_m1_epi.txt
: > $o
for k in 16 24 32; do
  echo "== K=$k KN_PIPE_EXACT=1" >> $o
  KN_PIPE_EXACT=1 timeout -k 10 150 python -u scripts/ab_tiles.py 900000 $k 7 100 base,_m1 >> $o 2>&1
  echo "== K=$k KN_PIPE_EXACT=0" >> $o
  KN_PIPE_EXACT=0 timeout -k 10 150 python -u scripts/ab_tiles.py 900000 $k 7 100 base,_m1 >> $o 2>&1
done
