#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5tblock
mkdir -p $O
run() { # name args...
  local name=$1; shift
  timeout -k 10 200 python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo FAIL $name; tail -5 $O/$name.err; exit 1; }
  echo "$name $(python -c "import json;d=json.loads(open('$O/$name.json').read().splitlines()[-1]);print(round(d['ms_per_step'],4), d.get('check',{}).get('bad_rows'), d.get('exact_path_queries'))")"
}
for rep in 1 2; do
  for b in 1 4 2; do
    export KN_TILE_BLOCK=$b
    run k16_b${b}_$rep --steps 200 --warmup 50 --no-check
    run m10_b${b}_$rep --n 10000000 --k 32 --steps 30 --warmup 10 --no-check
    run k50_b${b}_$rep --k 50 --steps 100 --warmup 30 --no-check
  done
done
export KN_TILE_BLOCK=4
run k16_b4_check --steps 20 --warmup 5
run m10_b4_check --n 10000000 --k 32 --steps 5 --warmup 2
