#!/bin/bash
# Round 6: re-rank group size after the in-order row stores (KN_RERANK_GROUP 8 default vs 4 / 16)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6group
mkdir -p $O
: > $O/ab.txt
for v in g4 g16; do
  for k in 50 32 64; do
    echo "== $v k=$k" >> $O/ab.txt
    timeout -k 10 200 python scripts/ab_variant.py $v 900000 $k 12 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $v $k"; exit 1; }
  done
done
cat $O/ab.txt
