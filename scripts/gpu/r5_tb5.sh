#!/bin/bash
# new size-dependent K<=16 tile order (default) vs the old fixed B=2 (KN_TILE_BLOCK=2); two passes,
# then the checked headline run
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5tb5
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
for V in new old; do
  E=KN_X=0; [ $V = old ] && E=KN_TILE_BLOCK=2
  one "$V 300K" $E -- --no-check --n 300000 --steps 200 --warmup 50
  one "$V 900K 200/50" $E -- --no-check --steps 200 --warmup 50
  one "$V 900K 20/5" $E -- --no-check --steps 20 --warmup 5
  one "$V 2M" $E -- --no-check --n 2000000 --steps 100 --warmup 30
  one "$V 4M" $E -- --no-check --n 4000000 --steps 60 --warmup 20
  one "$V 12.5M" $E -- --no-check --n 12500000 --steps 20 --warmup 10
done
done
one "new 300K check" KN_X=0 -- --n 300000 --steps 20 --warmup 5
one "new 4M check" KN_X=0 -- --n 4000000 --steps 10 --warmup 3
sort $O/ab.txt
