#!/bin/bash
# Lane-walk unroll 3 vs 2 at K=64 / 24 / 40 and a repeat at 16 / 32 (30 interleaved rounds).
set -o pipefail
export PYTHONPATH=$PWD
for k in 64 24 40 32 16 64; do
  echo "== unr3 K=$k"
  timeout -k 10 200 python scripts/ab_variant.py unr3 900000 $k 30 || { echo FAIL; exit 1; }
done
