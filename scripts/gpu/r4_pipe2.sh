#!/bin/bash
# Round 4: primed pipeline, trimmed events; unroll A/B at the driver's 20/5 and at 200/50.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4pipe2
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_tree.py \
  -k "pipelin or stream or relabel" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for rep in 1 2 3; do
  for u in 0 4 10; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --unroll $u > "$O/b20_u${u}_$rep.json" 2> "$O/b20_u${u}_$rep.err" || exit 1
    timeout -k 10 120 python3 bench.py --steps 200 --warmup 50 --unroll $u --no-check > "$O/b200_u${u}_$rep.json" 2> "$O/b200_u${u}_$rep.err" || exit 1
  done
done
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-check --stream-clouds 4 > "$O/stream20.json" 2> "$O/stream20.err" || exit 1
timeout -k 10 120 python3 bench.py --steps 200 --warmup 50 --stream-clouds 4 > "$O/stream200.json" 2> "$O/stream200.err" || exit 1
for f in "$O"/*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],4), d.get('check'))")"; done
