#!/bin/bash
# Round 4: forced-collective native pipeline, position-dependent halo (loopback 8 x 900K), GPU
# distributed tests, engine pipeline tests.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4dist2
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
KN_DIAG_VERBOSE=1 MASTER_PORT=$((29700 + RANDOM % 100)) timeout -k 10 120 python3 scripts/diag_dist_pipe.py 10 200000 > "$O/diag_pipe.log" 2>&1
rc=$?
grep -v "NCCL WARN\|^$" "$O/diag_pipe.log" | tail -12
[ $rc -eq 0 ] || { echo "diag_dist_pipe rc $rc"; exit 1; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py \
  > "$O/tests_dist.log" 2>&1 || { tail -40 "$O/tests_dist.log"; exit 1; }
tail -3 "$O/tests_dist.log"
for gen in uniform clustered; do
  timeout -k 10 300 python3 bench.py --loopback 8 --n 900000 --gen $gen --steps 10 --warmup 3 > "$O/loop8_$gen.json" 2> "$O/loop8_$gen.err" || { tail -20 "$O/loop8_$gen.err"; exit 1; }
  cat "$O/loop8_$gen.json"
done
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_tree.py \
  -k "pipelin or stream or relabel" > "$O/tests_pipe.log" 2>&1 || { tail -30 "$O/tests_pipe.log"; exit 1; }
tail -2 "$O/tests_pipe.log"
P=$((29800 + RANDOM % 100))
for mode in "" "--force-collectives"; do
  MASTER_PORT=$P timeout -k 10 180 python3 bench.py --dist $mode --steps 20 --warmup 5 > "$O/dist20${mode}.json" 2> "$O/dist20${mode}.err" || { tail -20 "$O/dist20${mode}.err"; exit 1; }
  P=$((P + 1))
  MASTER_PORT=$P timeout -k 10 180 python3 bench.py --dist $mode --steps 200 --warmup 50 --no-check > "$O/dist200${mode}.json" 2> "$O/dist200${mode}.err" || { tail -20 "$O/dist200${mode}.err"; exit 1; }
  P=$((P + 1))
done
for u in 0 4; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --unroll $u > "$O/b20_u${u}.json" 2> "$O/b20_u${u}.err" || exit 1
  timeout -k 10 120 python3 bench.py --steps 200 --warmup 50 --unroll $u --no-check > "$O/b200_u${u}.json" 2> "$O/b200_u${u}.err" || exit 1
done
for f in "$O"/dist*.json "$O"/b*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],4), d.get('check'), {k: d.get(k) for k in ('ms_route','ms_exchange','ms_build','ms_query','ms_finish','pipelined')})")"; done
