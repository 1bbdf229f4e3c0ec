#!/bin/bash
# Exact re-rank window kWin 2 / 4 vs 3 at K=16 / 50 (30 interleaved rounds).
set -o pipefail
export PYTHONPATH=$PWD
for v in win2 win4; do
  for k in 16 50; do
    echo "== $v K=$k"
    timeout -k 10 200 python scripts/ab_variant.py $v 900000 $k 30 || { echo FAIL; exit 1; }
  done
done
