#!/bin/bash
# tile-block order B=1 / 2 / 4 for K=16 across cloud sizes (is plain order better at 900K, and
# where does it stop paying?); two interleaved passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5tb4
mkdir -p $O
: > $O/ab.txt
one() {  # label env -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4))" >> $O/ab.txt
}
for pass in 1 2; do
for B in 1 2 4; do
  one "B=$B 300K" KN_TILE_BLOCK=$B -- --n 300000 --steps 200 --warmup 50
  one "B=$B 600K" KN_TILE_BLOCK=$B -- --n 600000 --steps 200 --warmup 50
  one "B=$B 900K 200/50" KN_TILE_BLOCK=$B -- --steps 200 --warmup 50
  one "B=$B 900K 20/5" KN_TILE_BLOCK=$B -- --steps 20 --warmup 5
  one "B=$B 2M" KN_TILE_BLOCK=$B -- --n 2000000 --steps 100 --warmup 30
  one "B=$B 4M" KN_TILE_BLOCK=$B -- --n 4000000 --steps 60 --warmup 20
  one "B=$B 900K k8" KN_TILE_BLOCK=$B -- --k 8 --steps 200 --warmup 50
done
done
sort $O/ab.txt
