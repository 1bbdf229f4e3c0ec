#!/bin/bash
# Round 6: narrower x halo (KN_XHALO_SUB=3 sub-cells = 1.5 cells; _C_hx3) vs 2 cells (_C): each with
# its own plan (scripts/ab_plan.py)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6hx
mkdir -p $O
: > $O/ab.txt
for n in 900000 300000 3000000; do
for k in 16 8; do
  echo "== hx3 n=$n k=$k" >> $O/ab.txt
  timeout -k 10 200 python scripts/ab_plan.py hx3 $n $k 14 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $n $k"; tail $O/ab.txt; exit 1; }
done
done
cat $O/ab.txt
