#!/bin/bash
# tile-block order B=1 vs 4 for K=50, 10M K=32, 12.5M K=16, clustered K=32 (grid fallback rows); two passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5tb3
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
for B in 1 4; do
  one "B=$B k50" KN_TILE_BLOCK=$B -- --k 50 --steps 100 --warmup 30
  one "B=$B k64" KN_TILE_BLOCK=$B -- --k 64 --steps 60 --warmup 20
  one "B=$B k24" KN_TILE_BLOCK=$B -- --k 24 --steps 100 --warmup 30
  one "B=$B 10M k32" KN_TILE_BLOCK=$B -- --n 10000000 --k 32 --steps 20 --warmup 10
  one "B=$B 12.5M k16" KN_TILE_BLOCK=$B -- --n 12500000 --k 16 --steps 20 --warmup 10
  one "B=$B 300K" KN_TILE_BLOCK=$B -- --n 300000 --steps 200 --warmup 50
done
done
sort $O/ab.txt
