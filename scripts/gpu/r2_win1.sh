#!/bin/bash
# Re-rank window kWin 1 vs the new default 2 at K=16 / 50 / 32 (30 interleaved rounds).
set -o pipefail
export PYTHONPATH=$PWD
for k in 16 50 32; do
  echo "== win1 K=$k"
  timeout -k 10 200 python scripts/ab_variant.py win1 900000 $k 30 || { echo FAIL; exit 1; }
done
