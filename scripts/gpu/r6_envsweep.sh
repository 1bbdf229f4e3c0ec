#!/bin/bash
# Round 6: run-time plan knobs re-checked at the headline (900K K=16, 200/50 steps) after the
# build / row-store changes: tile block order, x sub-cells, LDS slack
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6env
mkdir -p $O
: > $O/ab.txt
one() {  # label env args...
  local label=$1 ev=$2; shift 2
  env $ev timeout -k 10 120 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('ms_solve'))" >> $O/ab.txt
}
for pass in 1 2; do
  one "default" KN_X=0 --steps 200 --warmup 50
  one "tile_block=1" KN_TILE_BLOCK=1 --steps 200 --warmup 50
  one "tile_block=4" KN_TILE_BLOCK=4 --steps 200 --warmup 50
  one "xsub=1" KN_XSUB=1 --steps 200 --warmup 50
  one "lds_sd=4" KN_LDS_SD=4 --steps 200 --warmup 50
  one "lds_sd=6" KN_LDS_SD=6 --steps 200 --warmup 50
done
cat $O/ab.txt
