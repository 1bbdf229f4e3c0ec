#!/bin/bash
# Round 6: per-row staging with direct global->LDS loads (KN_STAGE_ROWS=1, _C) vs round 5 (_C_stage0)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6stage
mkdir -p $O
for c in "uniform 16" "uniform 50" "clustered 16"; do
  KN_CHECKED=1 timeout -k 10 120 python scripts/diag_engine_k.py $c > $O/chk_$(echo $c | tr ' ' _).txt 2>&1 || { echo "DIAG_FAIL checked $c"; tail -5 $O/chk_$(echo $c | tr ' ' _).txt; exit 1; }
  grep -v amdgpu.ids $O/chk_$(echo $c | tr ' ' _).txt | grep -E "debug_words|rows equal" | cut -c1-200
done
: > $O/ab.txt
for n in 900000 10000000; do
for k in 16 32 50; do
  if [ $n = 10000000 ] && [ $k != 32 ]; then continue; fi
  echo "== stage0 n=$n k=$k" >> $O/ab.txt
  timeout -k 10 200 python scripts/ab_variant.py stage0 $n $k 10 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $n $k"; tail $O/ab.txt; exit 1; }
done
done
echo "== stage0 n=300000 k=16" >> $O/ab.txt
timeout -k 10 200 python scripts/ab_variant.py stage0 300000 16 10 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL 300K"; exit 1; }
cat $O/ab.txt
