#!/bin/bash
# Re-rank window kWin 1 vs 3 at K=16/50, kWin 2 vs 3 at K=8/32/64 (30 interleaved rounds).
set -o pipefail
export PYTHONPATH=$PWD
for vk in "win1 16" "win1 50" "win2 8" "win2 32" "win2 64" "win2 16"; do
  set -- $vk
  echo "== $1 K=$2"
  timeout -k 10 200 python scripts/ab_variant.py $1 900000 $2 30 || { echo FAIL; exit 1; }
done
