#!/bin/bash
# Round 4: native pipeline loopback layouts at world > 1, RCCL world-1 diag with the eager
# warm-up, unroll A/B of the engine at the driver's 20/5.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4dist3
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py \
  -k "loopback_layouts or rccl_world1" > "$O/tests_dist.log" 2>&1 || { tail -40 "$O/tests_dist.log"; }
grep -E "PASS|FAIL" "$O/tests_dist.log" | tail -8
for rep in 1 2; do
  for u in 4 10 20; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --unroll $u --no-check > "$O/b20_u${u}_$rep.json" 2> "$O/b20_u${u}_$rep.err" || exit 1
  done
done
P=$((29800 + RANDOM % 100))
MASTER_PORT=$P timeout -k 10 180 python3 bench.py --dist --steps 200 --warmup 50 --no-check > "$O/dist200.json" 2> "$O/dist200.err" || { tail -20 "$O/dist200.err"; exit 1; }
MASTER_PORT=$((P+1)) timeout -k 10 180 python3 bench.py --dist --steps 20 --warmup 5 > "$O/dist20.json" 2> "$O/dist20.err" || { tail -20 "$O/dist20.err"; exit 1; }
timeout -k 10 120 python3 bench.py --steps 200 --warmup 50 --no-check > "$O/b200.json" 2> "$O/b200.err" || exit 1
for f in "$O"/*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],4), d.get('check'), {k: d.get(k) for k in ('ms_route','ms_exchange','ms_build','ms_query','ms_finish')})")"; done
for rep in 1 2; do
  for big in 0 1; do
    for k in 16 50; do
      KN_HOST_BIG=$big timeout -k 10 120 ./bin/knn_cli --uniform 900000 --k $k --api-bench 7 > "$O/api_big${big}_k${k}_$rep.json" 2> "$O/api_big${big}_k${k}_$rep.err" || { tail -5 "$O/api_big${big}_k${k}_$rep.err"; exit 1; }
    done
  done
done
cat "$O"/api_*.json
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_capi.py > "$O/tests_capi.log" 2>&1 || { tail -30 "$O/tests_capi.log"; exit 1; }
tail -2 "$O/tests_capi.log"
timeout -k 10 300 python3 scripts/ab_tiles.py 900000 16 5 100 > "$O/ab_tiles.log" 2>&1 || { tail -20 "$O/ab_tiles.log"; exit 1; }
timeout -k 10 300 python3 scripts/ab_tiles.py 900000 50 3 40 > "$O/ab_tiles50.log" 2>&1 || { tail -20 "$O/ab_tiles50.log"; exit 1; }
cat "$O/ab_tiles50.log"
cat "$O/ab_tiles.log"
timeout -k 10 2400 bash scripts/bench_suite.sh > "$O/suite.log" 2>&1 || { tail -20 "$O/suite.log"; exit 1; }
cp gpurun_out/bench_suite.jsonl "$O/bench_suite.jsonl"
tail -20 "$O/suite.log"
