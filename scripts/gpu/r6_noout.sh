#!/bin/bash
# Round 6 diagnostic: cost of the re-rank's per-entry row stores (_C_noout writes no rows)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6noout
mkdir -p $O
: > $O/ab.txt
for k in 16 50 32; do
  echo "== noout k=$k" >> $O/ab.txt
  timeout -k 10 200 python scripts/ab_variant.py noout 900000 $k 14 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $k"; exit 1; }
done
cat $O/ab.txt
