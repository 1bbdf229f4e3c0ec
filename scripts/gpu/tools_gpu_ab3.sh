#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/ab3.log
: > $O
timeout -k 10 120 python scripts/ab_variant.py pipechk 100000 16 2 >> $O 2>&1 || { echo CHK_FAIL; tail -5 $O; exit 1; }
for v in pipe pipeypr ypr; do
  timeout -k 10 120 python scripts/ab_variant.py $v 900000 16 15 >> $O 2>&1 || { echo AB_FAIL $v; tail -5 $O; exit 1; }
done
timeout -k 10 120 python scripts/ab_variant.py pipeypr 900000 32 8 >> $O 2>&1 || { echo AB32_FAIL; tail -5 $O; exit 1; }
timeout -k 10 120 python scripts/ab_variant.py pipeypr 900000 50 6 >> $O 2>&1 || { echo AB50_FAIL; tail -5 $O; exit 1; }
grep -v amdgpu.ids $O
