#!/bin/bash
# Round 6: gated-tier top-K networks (KN_TOPK_TIERS) vs the single network, in-process A/B
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6ab2
mkdir -p $O
: > $O/ab.txt
for k in 16 50 32 8 64; do
  for var in tiers2 tiers3 tiers4; do
    echo "== $var k=$k" >> $O/ab.txt
    timeout -k 10 150 python scripts/ab_variant.py $var 900000 $k 10 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $var $k"; tail $O/ab.txt; exit 1; }
  done
done
cat $O/ab.txt
