#!/bin/bash
# Round 4: full GPU tests (halo field, lane-walk margin 1 above K=32, route-count ballots, THP
# getter copy-out), loopback halo fractions with the field, API host-to-host bench, headline /
# distributed / K=50 benches.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4ab6
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
for g in uniform clustered; do
  timeout -k 10 300 python3 bench.py --loopback 8 --n 900000 --gen $g --steps 10 --warmup 3 > "$O/lb_$g.json" 2> "$O/lb_$g.err" || { tail -20 "$O/lb_$g.err"; exit 1; }
  KN_HALO_FIELD_G=0 timeout -k 10 300 python3 bench.py --loopback 8 --n 900000 --gen $g --steps 10 --warmup 3 > "$O/lb_${g}_nofield.json" 2> "$O/lb_${g}_nofield.err" || { tail -20 "$O/lb_${g}_nofield.err"; exit 1; }
done
for f in "$O"/lb_*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],3), d['check'], {k: d['stats'].get(k) for k in ('halo_frac_max','halo_width','halo_field','forwarded','steady')})")"; done
for k in 16 50; do
  timeout -k 10 120 ./bin/knn_cli --uniform 900000 --k $k --api-bench 7 > "$O/api_k$k.json" 2> "$O/api_k$k.err" || { tail -5 "$O/api_k$k.err"; exit 1; }
  KN_HOST_BIG=0 timeout -k 10 120 ./bin/knn_cli --uniform 900000 --k $k --api-bench 7 > "$O/api_k${k}_big0.json" 2> "$O/api_k${k}_big0.err" || { tail -5 "$O/api_k${k}_big0.err"; exit 1; }
done
cat "$O"/api_*.json
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > "$O/b20.json" 2> "$O/b20.err" || exit 1
timeout -k 10 120 python3 bench.py --steps 200 --warmup 50 --no-check > "$O/b200.json" 2> "$O/b200.err" || exit 1
timeout -k 10 120 python3 bench.py --k 50 --steps 100 --warmup 30 > "$O/b50.json" 2> "$O/b50.err" || exit 1
P=$((29800 + RANDOM % 100))
MASTER_PORT=$P timeout -k 10 180 python3 bench.py --dist --steps 20 --warmup 5 > "$O/d20.json" 2> "$O/d20.err" || { tail -20 "$O/d20.err"; exit 1; }
MASTER_PORT=$((P+1)) timeout -k 10 180 python3 bench.py --dist --steps 200 --warmup 50 --no-check > "$O/d200.json" 2> "$O/d200.err" || { tail -20 "$O/d200.err"; exit 1; }
for f in "$O"/b*.json "$O"/d*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],4), d.get('check'), d.get('exact_path_queries'), {k: d.get(k) for k in ('ms_route','ms_build','ms_query','ms_finish')})")"; done
cd /tmp
MASTER_PORT=$((29700 + RANDOM % 100)) timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$O/trace_dist" -o run -- python3 "$R/bench.py" --dist --steps 20 --warmup 5 --no-check > "$O/trace_dist.log" 2>&1 || { tail -20 "$O/trace_dist.log"; exit 1; }
