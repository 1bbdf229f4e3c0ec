#!/bin/bash
# K=50 knobs under the round-5 pipeline: tile-block size, x sub-cells, LDS slack; 100 / 30, two passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5k50b
mkdir -p $O
: > $O/ab.txt
one() {  # label env...
  local label=$1; shift
  env "$@" timeout -k 10 150 python bench.py --no-check --k 50 --steps 100 --warmup 30 > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('exact_path_queries'), d.get('grid'))" >> $O/ab.txt
}
for pass in 1 2; do
  one "base"
  one "tblock2" KN_TILE_BLOCK=2
  one "tblock8" KN_TILE_BLOCK=8
  one "xsub2" KN_XSUB=2
  one "ldssd3" KN_LDS_SD=3
  one "ldssd7" KN_LDS_SD=7
done
sort $O/ab.txt
