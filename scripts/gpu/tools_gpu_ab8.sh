#!/bin/bash
# KN_LANE_UNROLL 3/4 vs 2 at K=50/64 (3-ring-halo plans) and K=32
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/ab8.log
: > $O
for v in u4 u3; do
  for k in 50 64 32; do
    echo "== $v k=$k" >> $O
    timeout -k 10 120 python scripts/ab_variant.py $v 900000 $k 10 >> $O 2>&1 || { echo AB_FAIL $v $k; tail -5 $O; exit 1; }
  done
done
grep -v amdgpu $O
