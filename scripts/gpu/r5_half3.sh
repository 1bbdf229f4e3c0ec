#!/bin/bash
# 4x2x4 tiles below 1,500 rounded 4^3 tiles (default) vs never (KN_HALF_TILE_MAX=0); two passes, checks
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5half3
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
  E=KN_X=0; [ $V = old ] && E=KN_HALF_TILE_MAX=0
  for n in 100000 150000 250000 300000 320000; do
    one "$V $n" $E -- --no-check --n $n --steps 200 --warmup 50
  done
  one "$V 250000 k50" $E -- --no-check --k 50 --n 250000 --steps 100 --warmup 30
done
done
for n in 100000 150000 250000 320000; do one "new $n check" KN_X=0 -- --n $n --steps 20 --warmup 5; done
one "new 250000 k50 check" KN_X=0 -- --k 50 --n 250000 --steps 20 --warmup 5
sort $O/ab.txt
