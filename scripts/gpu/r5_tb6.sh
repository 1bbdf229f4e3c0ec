#!/bin/bash
# K=32 tile order B=1 vs 4 away from 900K, and K=8 at 300K / 4M (B 1 / 2 / 4); two passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5tb6
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
  one "B=$B k32 300K" KN_TILE_BLOCK=$B -- --k 32 --n 300000 --steps 200 --warmup 50
  one "B=$B k32 2M" KN_TILE_BLOCK=$B -- --k 32 --n 2000000 --steps 100 --warmup 30
  one "B=$B k32 4M" KN_TILE_BLOCK=$B -- --k 32 --n 4000000 --steps 60 --warmup 20
  one "B=$B k8 300K" KN_TILE_BLOCK=$B -- --k 8 --n 300000 --steps 200 --warmup 50
  one "B=$B k8 4M" KN_TILE_BLOCK=$B -- --k 8 --n 4000000 --steps 60 --warmup 20
  one "B=$B k24 900K" KN_TILE_BLOCK=$B -- --k 24 --steps 100 --warmup 30
done
done
sort $O/ab.txt
