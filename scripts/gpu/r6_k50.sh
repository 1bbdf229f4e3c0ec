#!/bin/bash
# Round 6: K=50 bucket -- walk unroll 2 (u50x2), re-rank groups of 8 (grp8), 4 tiers (t50x4, all K>40:
# also forces K=16 to 4 tiers, so only the K=50 / 64 rows count) vs the defaults
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6k50
mkdir -p $O
: > $O/ab.txt
for var in u50x2 grp8 t50x4; do
for k in 50 64; do
  echo "== $var k=$k" >> $O/ab.txt
  timeout -k 10 200 python scripts/ab_variant.py $var 900000 $k 14 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $var $k"; tail $O/ab.txt; exit 1; }
done
done
cat $O/ab.txt
