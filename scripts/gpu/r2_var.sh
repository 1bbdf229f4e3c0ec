#!/bin/bash
# In-process A/B of kernel variants: row-wise staging (KN_STAGE_ROWS=1), lane-walk unroll 1.
set -o pipefail
export PYTHONPATH=$PWD
for v in rows unr1; do
  for k in 16 50; do
    echo "== $v K=$k"
    timeout -k 10 200 python scripts/ab_variant.py $v 900000 $k 15 || { echo FAIL $v $k; exit 1; }
  done
done
