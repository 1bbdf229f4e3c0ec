#!/bin/bash
# A/B of query-kernel variants vs the default build (_C), query kernel only, interleaved in
# process (scripts/ab_variant.py): slow = the correctly rounded sqrtf + the old cell_coord;
# split1 / split2 = split top-K networks; rrun = unrolled re-rank (KM <= 24).
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5split
mkdir -p $O
for k in 16 50; do
  for v in slow split1 split2 rrun; do
    echo "k=$k $v: $(timeout -k 10 120 python scripts/ab_variant.py $v 900000 $k 15 2>&1 | tr '\n' ' ')"
  done
done | tee $O/ab.txt
for k in 8 32 64; do
  for v in slow split2; do
    echo "k=$k $v: $(timeout -k 10 120 python scripts/ab_variant.py $v 900000 $k 15 2>&1 | tr '\n' ' ')"
  done
done | tee -a $O/ab.txt
