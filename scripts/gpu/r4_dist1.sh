#!/bin/bash
# Round 4: native distributed pipeline at world 1 (RCCL) + the engine pipeline A/B.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4dist1
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py \
  -k "rccl_world1" > "$O/tests_dist.log" 2>&1 || { tail -40 "$O/tests_dist.log"; exit 1; }
tail -4 "$O/tests_dist.log"
P=$((29600 + RANDOM % 200))
for mode in "" "--force-collectives"; do
  for rep in 1 2; do
    MASTER_PORT=$P timeout -k 10 180 python3 bench.py --dist $mode --steps 20 --warmup 5 > "$O/dist20${mode}_$rep.json" 2> "$O/dist20${mode}_$rep.err" || { tail -20 "$O/dist20${mode}_$rep.err"; exit 1; }
    P=$((P + 1))
    MASTER_PORT=$P timeout -k 10 180 python3 bench.py --dist $mode --steps 200 --warmup 50 --no-check > "$O/dist200${mode}_$rep.json" 2> "$O/dist200${mode}_$rep.err" || { tail -20 "$O/dist200${mode}_$rep.err"; exit 1; }
    P=$((P + 1))
  done
done
for rep in 1 2; do
  for u in 0 4; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --unroll $u > "$O/b20_u${u}_$rep.json" 2> "$O/b20_u${u}_$rep.err" || exit 1
    timeout -k 10 120 python3 bench.py --steps 200 --warmup 50 --unroll $u --no-check > "$O/b200_u${u}_$rep.json" 2> "$O/b200_u${u}_$rep.err" || exit 1
  done
done
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-check --stream-clouds 4 > "$O/stream20.json" 2> "$O/stream20.err" || exit 1
for f in "$O"/*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],4), d.get('check'), {k: d.get(k) for k in ('ms_route','ms_exchange','ms_build','ms_query','ms_flag_allreduce','pipelined')})")"; done
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_tree.py \
  -k "pipelin or stream or relabel" > "$O/tests_pipe.log" 2>&1 || { tail -30 "$O/tests_pipe.log"; exit 1; }
tail -2 "$O/tests_pipe.log"
