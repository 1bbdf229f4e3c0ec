#!/bin/bash
# Round 4: host copy probe (DMA split / kernel copies), full GPU tests after the route-count and
# top-K margin changes, headline / distributed / K=50 benches.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4ab5
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
timeout -k 10 120 ./bin/hostio_probe 61.2 5 > "$O/hostio_k16.jsonl" 2> "$O/hostio.err" || { cat "$O/hostio.err"; exit 1; }
head -8 "$O/hostio_k16.jsonl"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > "$O/b20.json" 2> "$O/b20.err" || exit 1
timeout -k 10 120 python3 bench.py --steps 200 --warmup 50 --no-check > "$O/b200.json" 2> "$O/b200.err" || exit 1
timeout -k 10 120 python3 bench.py --k 50 --steps 100 --warmup 30 > "$O/b50.json" 2> "$O/b50.err" || exit 1
P=$((29800 + RANDOM % 100))
MASTER_PORT=$P timeout -k 10 180 python3 bench.py --dist --steps 20 --warmup 5 > "$O/d20.json" 2> "$O/d20.err" || { tail -20 "$O/d20.err"; exit 1; }
MASTER_PORT=$((P+1)) timeout -k 10 180 python3 bench.py --dist --steps 200 --warmup 50 --no-check > "$O/d200.json" 2> "$O/d200.err" || { tail -20 "$O/d200.err"; exit 1; }
for f in "$O"/*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],4), d.get('check'), d.get('exact_path_queries'), {k: d.get(k) for k in ('ms_route','ms_build','ms_query','ms_finish')})")"; done
cd /tmp
MASTER_PORT=$((29700 + RANDOM % 100)) timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$O/trace_dist" -o run -- python3 "$R/bench.py" --dist --steps 20 --warmup 5 --no-check > "$O/trace_dist.log" 2>&1 || { tail -20 "$O/trace_dist.log"; exit 1; }
