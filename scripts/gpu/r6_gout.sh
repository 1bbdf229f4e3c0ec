#!/bin/bash
# Round 6: global-address-space output stores (KN_GLOBAL_OUT=1, _C) vs generic/FLAT (_C_gout0)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6gout
mkdir -p $O
: > $O/ab.txt
for k in 16 50 32 8; do
  echo "== gout0 k=$k" >> $O/ab.txt
  timeout -k 10 200 python scripts/ab_variant.py gout0 900000 $k 12 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $k"; tail $O/ab.txt; exit 1; }
done
echo "== tree gout0 k=16" >> $O/ab.txt
timeout -k 10 300 python scripts/ab_tree.py _gout0 4 20 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "ABTREE_FAIL"; tail $O/ab.txt; exit 1; }
cat $O/ab.txt
