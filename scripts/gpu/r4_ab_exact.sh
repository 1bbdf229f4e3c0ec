#!/bin/bash
# Round 4: exact finish in the query stage (KN_PIPE_EXACT=0) vs as the build-stream epilogue (1),
# interleaved on one box; world-1 distributed step; one clean JSON line on stdout.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4abx
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
for rep in 1 2 3; do
  for x in 0 1; do
    KN_PIPE_EXACT=$x timeout -k 10 120 python3 bench.py --steps 200 --warmup 50 --no-check > "$O/b200_x${x}_$rep.json" 2> "$O/b200_x${x}_$rep.err" || exit 1
    KN_PIPE_EXACT=$x timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 > "$O/b20_x${x}_$rep.json" 2> "$O/b20_x${x}_$rep.err" || exit 1
  done
done
P=$((29800 + RANDOM % 100))
MASTER_PORT=$P timeout -k 10 180 python3 bench.py --dist --steps 200 --warmup 50 --no-check > "$O/dist200.json" 2> "$O/dist200.err" || { tail -20 "$O/dist200.err"; exit 1; }
MASTER_PORT=$((P + 1)) timeout -k 10 180 python3 bench.py --dist --steps 20 --warmup 5 > "$O/dist20.json" 2> "$O/dist20.err" || { tail -20 "$O/dist20.err"; exit 1; }
for f in "$O"/*.json; do echo "$(basename $f) $(wc -l < $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],4), d.get('check'), {k: d.get(k) for k in ('ms_route','ms_exchange','ms_build','ms_query','ms_finish')})")"; done
