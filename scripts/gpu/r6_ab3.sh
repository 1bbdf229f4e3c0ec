#!/bin/bash
# Round 6: grouped re-rank walk (KN_RERANK_GROUP, baseline 4) vs 1 / 2 / 8 on the rolled K buckets,
# and gated tiers in the tree query (K=50 / 64, clustered + surface)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6ab3
mkdir -p $O
: > $O/ab.txt
for k in 32 50 64; do
  for var in grp1 grp2 grp8; do
    echo "== $var k=$k" >> $O/ab.txt
    timeout -k 10 150 python scripts/ab_variant.py $var 900000 $k 10 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $var $k"; tail $O/ab.txt; exit 1; }
  done
done
for k in 50 64; do
  echo "== tree ttiers k=$k" >> $O/ab.txt
  AB_K=$k timeout -k 10 300 python scripts/ab_tree.py _ttiers 4 20 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "ABTREE_FAIL $k"; tail $O/ab.txt; exit 1; }
done
cat $O/ab.txt
