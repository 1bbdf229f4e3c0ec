#!/bin/bash
# Round 3 lane-walk A/B: fast re-rank, pipelined gathers, R-capped bound, all three; SLP build.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/ab1
mkdir -p $O
for v in fast pipe rcap all slp; do
  timeout -k 10 200 python scripts/ab_multi.py $v 900000 8,16,32,50,64 uniform 10 > $O/$v.jsonl 2>> $O/err.log || { echo AB_FAIL $v; tail -20 $O/err.log; exit 1; }
  cat $O/$v.jsonl
done
# host-to-host reference API (kn_prepare from host -> kn_solve -> getters), K=16 and K=50
timeout -k 10 200 ./bin/knn_cli --uniform 900000 --k 16 --api-bench 5 > $O/api16.json 2>> $O/err.log || { echo API_FAIL; tail $O/err.log; exit 1; }
cat $O/api16.json
timeout -k 10 200 ./bin/knn_cli --uniform 900000 --k 50 --api-bench 5 > $O/api50.json 2>> $O/err.log || { echo API_FAIL; tail $O/err.log; exit 1; }
cat $O/api50.json
