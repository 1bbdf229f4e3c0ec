#!/bin/bash
# Round 4: host getter probe, tile/margin A/B (module-local bindings), unroll A/B of the engine
# and the distributed pipeline, kernel traces of the native and distributed 20/5 runs.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4ab4
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
timeout -k 10 120 ./bin/hostio_probe 61.2 5 > "$O/hostio_k16.jsonl" 2> "$O/hostio.err" || { cat "$O/hostio.err"; exit 1; }
timeout -k 10 120 ./bin/hostio_probe 183.6 3 > "$O/hostio_k50.jsonl" 2>> "$O/hostio.err" || { cat "$O/hostio.err"; exit 1; }
cat "$O/hostio_k16.jsonl"
timeout -k 10 300 python3 scripts/ab_tiles.py 900000 16 5 100 > "$O/ab_tiles.log" 2>&1 || { tail -20 "$O/ab_tiles.log"; exit 1; }
timeout -k 10 300 python3 scripts/ab_tiles.py 900000 50 3 40 > "$O/ab_tiles50.log" 2>&1 || { tail -20 "$O/ab_tiles50.log"; exit 1; }
grep median "$O/ab_tiles.log" "$O/ab_tiles50.log"
for rep in 1 2; do
  for u in 4 10; do
    timeout -k 10 120 python3 bench.py --steps 200 --warmup 50 --unroll $u --no-check > "$O/b200_u${u}_$rep.json" 2> "$O/b200_u${u}_$rep.err" || exit 1
    P=$((29800 + RANDOM % 100))
    KN_DIST_UNROLL=$u MASTER_PORT=$P timeout -k 10 180 python3 bench.py --dist --steps 20 --warmup 5 --no-check > "$O/d20_u${u}_$rep.json" 2> "$O/d20_u${u}_$rep.err" || { tail -20 "$O/d20_u${u}_$rep.err"; exit 1; }
    KN_DIST_UNROLL=$u MASTER_PORT=$((P+1)) timeout -k 10 180 python3 bench.py --dist --steps 200 --warmup 50 --no-check > "$O/d200_u${u}_$rep.json" 2> "$O/d200_u${u}_$rep.err" || { tail -20 "$O/d200_u${u}_$rep.err"; exit 1; }
  done
done
for f in "$O"/*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],4))")"; done
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$O/trace_native" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-check > "$O/trace_native.log" 2>&1 || { tail -20 "$O/trace_native.log"; exit 1; }
MASTER_PORT=$((29700 + RANDOM % 100)) timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$O/trace_dist" -o run -- python3 "$R/bench.py" --dist --steps 20 --warmup 5 --no-check > "$O/trace_dist.log" 2>&1 || { tail -20 "$O/trace_dist.log"; exit 1; }
find "$O" -name "*kernel_trace.csv" | xargs ls -la
