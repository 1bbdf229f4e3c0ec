#!/bin/bash
# Round 4: GPU tests (default: three-kernel steady router), the refill diagnostics of the fused
# router, and the distributed bench with both routers.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4ab7
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
MODES=1,1 KN_ROUTE_FUSED=1 MASTER_PORT=$((29600 + RANDOM % 300)) timeout -k 10 200 python3 scripts/diag_dist_pipe.py 30 200000 1,1 > "$O/diag_11.log" 2>&1; grep -E "refill|ALL OK|FAILED" "$O/diag_11.log" | tail -3
KN_ROUTE_FUSED=1 KN_ARENA_CACHE=0 MASTER_PORT=$((29600 + RANDOM % 300)) timeout -k 10 200 python3 scripts/diag_dist_pipe.py 30 200000 0,1 > "$O/diag_01_nocache.log" 2>&1; grep -E "refill|ALL OK|FAILED" "$O/diag_01_nocache.log" | tail -3
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
for fused in 0 1; do
  P=$((29800 + RANDOM % 100))
  KN_ROUTE_FUSED=$fused MASTER_PORT=$P timeout -k 10 180 python3 bench.py --dist --steps 20 --warmup 5 > "$O/d20_f$fused.json" 2> "$O/d20_f$fused.err" || { tail -20 "$O/d20_f$fused.err"; exit 1; }
  KN_ROUTE_FUSED=$fused MASTER_PORT=$((P+1)) timeout -k 10 180 python3 bench.py --dist --steps 200 --warmup 50 --no-check > "$O/d200_f$fused.json" 2> "$O/d200_f$fused.err" || { tail -20 "$O/d200_f$fused.err"; exit 1; }
done
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > "$O/b20.json" 2> "$O/b20.err" || exit 1
timeout -k 10 120 python3 bench.py --steps 200 --warmup 50 --no-check > "$O/b200.json" 2> "$O/b200.err" || exit 1
timeout -k 10 120 python3 bench.py --k 50 --steps 100 --warmup 30 > "$O/b50.json" 2> "$O/b50.err" || exit 1
for f in "$O"/*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],4), d.get('check'), d.get('exact_path_queries'), {k: d.get(k) for k in ('ms_route','ms_build','ms_query','ms_finish')})")"; done
for g in uniform clustered; do
  timeout -k 10 300 python3 bench.py --loopback 8 --n 900000 --gen $g --steps 10 --warmup 3 > "$O/lb_$g.json" 2> "$O/lb_$g.err" || { tail -20 "$O/lb_$g.err"; exit 1; }
done
for f in "$O"/lb_*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],3), d['check'], {k: d['stats'].get(k) for k in ('halo_frac_max','halo_width','halo_field','forwarded','steady')})")"; done
for k in 16 50; do
  timeout -k 10 120 ./bin/knn_cli --uniform 900000 --k $k --api-bench 7 > "$O/api_k$k.json" 2> "$O/api_k$k.err" || { tail -5 "$O/api_k$k.err"; exit 1; }
done
cat "$O"/api_*.json
