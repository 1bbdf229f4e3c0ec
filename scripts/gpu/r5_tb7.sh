#!/bin/bash
# size-dependent tile order (default) vs the previous defaults (K=32: B=1 up to 4M; K<=16: B=2);
# two passes, then checked runs
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5tb7
mkdir -p $O
: > $O/ab.txt
one() {  # label env -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('check'))" >> $O/ab.txt
}
for pass in 1 2; do
  one "new k32 300K" KN_X=0 -- --no-check --k 32 --n 300000 --steps 200 --warmup 50
  one "old k32 300K" KN_TILE_BLOCK=1 -- --no-check --k 32 --n 300000 --steps 200 --warmup 50
  one "new k32 900K" KN_X=0 -- --no-check --k 32 --steps 100 --warmup 30
  one "old k32 900K" KN_TILE_BLOCK=1 -- --no-check --k 32 --steps 100 --warmup 30
  one "new k32 4M" KN_X=0 -- --no-check --k 32 --n 4000000 --steps 60 --warmup 20
  one "old k32 4M" KN_TILE_BLOCK=1 -- --no-check --k 32 --n 4000000 --steps 60 --warmup 20
  one "new k8 300K" KN_X=0 -- --no-check --k 8 --n 300000 --steps 200 --warmup 50
  one "old k8 300K" KN_TILE_BLOCK=2 -- --no-check --k 8 --n 300000 --steps 200 --warmup 50
done
one "new k32 300K check" KN_X=0 -- --k 32 --n 300000 --steps 20 --warmup 5
one "new k32 4M check" KN_X=0 -- --k 32 --n 4000000 --steps 10 --warmup 3
one "new k8 300K check" KN_X=0 -- --k 8 --n 300000 --steps 20 --warmup 5
sort $O/ab.txt
