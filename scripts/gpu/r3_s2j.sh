#!/bin/bash
# Round 3 (session 2): grouped tree traversal (G = 4 / 2 groups per wave) vs the wave-wide one.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2j
mkdir -p $O
for v in tg4 tg2; do
  timeout -k 10 400 python scripts/ab_tree.py $v 900000 16,50 clustered,surface,uniform 6 > $O/ab_$v.jsonl 2>> $O/err.log || { echo AB_FAIL $v; tail -20 $O/err.log; cat $O/ab_$v.jsonl; exit 1; }
  cat $O/ab_$v.jsonl
done
