#!/bin/bash
# workgroup tile-block order (KN_TILE_BLOCK) under the final pipeline, K=16 / K=32; two passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5tb2
mkdir -p $O
: > $O/ab.txt
one() {  # label env -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 150 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4))" >> $O/ab.txt
}
for pass in 1 2; do
for B in 1 2 4; do
  one "B=$B k16 200/50" KN_TILE_BLOCK=$B -- --steps 200 --warmup 50
  one "B=$B k16 20/5" KN_TILE_BLOCK=$B -- --steps 20 --warmup 5
  one "B=$B k32" KN_TILE_BLOCK=$B -- --k 32 --steps 100 --warmup 30
done
done
sort $O/ab.txt
