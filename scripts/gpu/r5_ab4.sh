#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5ab4
mkdir -p $O
for k in 50 64 16; do
  echo "k=$k slow: $(timeout -k 10 120 python scripts/ab_variant.py slow 900000 $k 20 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')"
done | tee $O/ab.txt
bash scripts/gpu/r5_qs_dbg.sh
