#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/ab2.log
: > $O
timeout -k 10 120 python scripts/ab_variant.py bothchk 100000 16 2 >> $O 2>&1 || { echo CHK_FAIL; tail -5 $O; exit 1; }
for v in rows ypr both; do
  timeout -k 10 120 python scripts/ab_variant.py $v 900000 16 12 >> $O 2>&1 || { echo AB_FAIL $v; tail -5 $O; exit 1; }
done
timeout -k 10 120 python scripts/ab_variant.py both 900000 32 8 >> $O 2>&1 || { echo AB32_FAIL; tail -5 $O; exit 1; }
grep -v amdgpu.ids $O
