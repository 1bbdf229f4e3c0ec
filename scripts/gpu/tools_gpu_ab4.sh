#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/ab4.log
: > $O
timeout -k 10 120 python scripts/ab_variant.py pairschk 100000 16 2 >> $O 2>&1 || { echo CHK_FAIL; tail -5 $O; exit 1; }
timeout -k 10 120 python scripts/ab_variant.py pairschk 60000 50 2 >> $O 2>&1 || { echo CHK2_FAIL; tail -5 $O; exit 1; }
for k in 16 8 32 50; do
  timeout -k 10 120 python scripts/ab_variant.py pairs 900000 $k 12 >> $O 2>&1 || { echo AB_FAIL $k; tail -5 $O; exit 1; }
done
cat $O | grep -v amdgpu.ids
