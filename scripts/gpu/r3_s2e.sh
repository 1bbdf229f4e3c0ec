#!/bin/bash
# Round 3 (session 2): packed outer rows A/B (_C vs _C_opack), host API with the block cache
# on / off (staging off).
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2e
mkdir -p $O
timeout -k 10 300 python scripts/ab_multi.py opack 900000 8,16,24,32,40 uniform 12 > $O/ab_opack.jsonl 2>> $O/err.log || { echo AB_FAIL; tail -20 $O/err.log; exit 1; }
timeout -k 10 300 python scripts/ab_multi.py opack 900000 16 blue,clustered 8 >> $O/ab_opack.jsonl 2>> $O/err.log || { echo AB2_FAIL; tail -20 $O/err.log; exit 1; }
timeout -k 10 300 python scripts/ab_multi.py opack 100000 8,16 uniform 12 >> $O/ab_opack.jsonl 2>> $O/err.log || { echo AB3_FAIL; tail -20 $O/err.log; exit 1; }
cat $O/ab_opack.jsonl
for c in 0 1; do
  KN_ARENA_CACHE=$c timeout -k 10 200 ./bin/knn_cli --uniform 900000 --k 16 --api-bench 7 > $O/api16_c$c.json 2> $O/api16_c$c.log || { echo API_FAIL; tail $O/api16_c$c.log; exit 1; }
  echo "cache=$c $(cat $O/api16_c$c.json)"
done
