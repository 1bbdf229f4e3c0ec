#!/bin/bash
# half-tile cut at 2000 4^3 tiles: 350K (1,728 tiles: halved) / 400K, 450K (2,197: 4^3) vs KN_HALF_TILE_MAX=0
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5half2
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
  one "$V 350K" $E -- --no-check --n 350000 --steps 200 --warmup 50
  one "$V 400K" $E -- --no-check --n 400000 --steps 200 --warmup 50
  one "$V 300K" $E -- --no-check --n 300000 --steps 200 --warmup 50
done
done
one "new 350K check" KN_X=0 -- --n 350000 --steps 20 --warmup 5
sort $O/ab.txt
