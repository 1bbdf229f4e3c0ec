#!/bin/bash
# Round 6: lane-walk gathers in flight re-checked after the round-6 kernel changes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6unroll
mkdir -p $O
: > $O/ab.txt
for spec in "u40x4 16" "u40x4 8" "u40x4 32" "u40x2 16" "u40x2 32" "u64x1 64" "u64x3 64"; do
  set -- $spec
  echo "== $1 k=$2" >> $O/ab.txt
  timeout -k 10 200 python scripts/ab_variant.py $1 900000 $2 14 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $spec"; exit 1; }
done
cat $O/ab.txt
