#!/bin/bash
# Round 6: K=64 register cap re-check after the row-store change (KN_TILE_WPE64=4 default: 128
# VGPRs with spills, vs 1: no cap, 3 workgroups per CU)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6wpe
mkdir -p $O
: > $O/ab.txt
for k in 64 64; do
  echo "== wpe1 k=$k" >> $O/ab.txt
  timeout -k 10 200 python scripts/ab_variant.py wpe1 900000 $k 14 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $k"; exit 1; }
done
cat $O/ab.txt
