#!/bin/bash
# 4x2x4 tiles for clouds of < 2400 4^3 tiles (default) vs always 4^3 (KN_HALF_TILE_MAX=0); two passes,
# then checked runs
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5half
mkdir -p $O
: > $O/ab.txt
one() {  # label env -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('check'), d.get('exact_path_queries'))" >> $O/ab.txt
}
for pass in 1 2; do
for V in new old; do
  E=KN_X=0; [ $V = old ] && E=KN_HALF_TILE_MAX=0
  one "$V 200K" $E -- --no-check --n 200000 --steps 200 --warmup 50
  one "$V 300K" $E -- --no-check --n 300000 --steps 200 --warmup 50
  one "$V 450K" $E -- --no-check --n 450000 --steps 200 --warmup 50
  one "$V 300K k32" $E -- --no-check --k 32 --n 300000 --steps 200 --warmup 50
  one "$V 300K k50" $E -- --no-check --k 50 --n 300000 --steps 100 --warmup 30
  one "$V 300K k8" $E -- --no-check --k 8 --n 300000 --steps 200 --warmup 50
  one "$V 900K" $E -- --no-check --steps 20 --warmup 5
done
done
for n in 200000 300000 450000; do one "new $n check" KN_X=0 -- --n $n --steps 20 --warmup 5; done
one "new 300K k50 check" KN_X=0 -- --k 50 --n 300000 --steps 20 --warmup 5
one "new 300K k64 check" KN_X=0 -- --k 64 --n 300000 --steps 20 --warmup 5
sort $O/ab.txt
