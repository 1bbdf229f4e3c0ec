#!/bin/bash
# In-process A/B: top-K margin M=3 (_C_m3) vs the default M=2, K=16 / 32 / 50.
set -o pipefail
export PYTHONPATH=$PWD
for k in 16 32 50; do
  timeout -k 10 200 python scripts/ab_variant.py m3 900000 $k 15 || { echo FAIL $k; exit 1; }
done
