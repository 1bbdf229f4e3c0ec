#!/bin/bash
# Round 6: in-process A/B of query-kernel variants (scripts/ab_variant.py: _C vs _C_<var>, rows
# must be identical), then the capture-crash probes of r6_c.sh
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6ab1
mkdir -p $O
for var in nopair runroll; do
  for k in 16 32 8; do
    echo "== $var k=$k" | tee -a $O/ab.txt
    timeout -k 10 120 python scripts/ab_variant.py $var 900000 $k 12 >> $O/ab.txt 2>&1 || { echo "AB_FAIL $var $k"; tail $O/ab.txt; exit 1; }
  done
done
cat $O/ab.txt
bash scripts/gpu/r6_c.sh
