#!/bin/bash
# Lane-walk unroll 1 vs 2 at K=50 / 64 (30 interleaved rounds, twice).
set -o pipefail
export PYTHONPATH=$PWD
for k in 50 64 50 64; do
  echo "== unr1 K=$k"
  timeout -k 10 200 python scripts/ab_variant.py unr1 900000 $k 30 || { echo FAIL; exit 1; }
done
