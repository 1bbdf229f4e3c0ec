#!/bin/bash
# Large clouds: workgroup tile-block size (KN_TILE_BLOCK) sweep, 10M K=32 and 12.5M K=16, pipelined
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5bigtb
mkdir -p $O
: > $O/ab.txt
one() {  # label args...
  local label=$1; shift
  timeout -k 10 200 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4))" >> $O/ab.txt
}
for pass in 1 2; do
for b in 2 4 8; do
  KN_TILE_BLOCK=$b one "10M k32 B=$b" --n 10000000 --k 32 --steps 20 --warmup 10
  KN_TILE_BLOCK=$b one "12.5M k16 B=$b" --n 12500000 --k 16 --steps 20 --warmup 10
done
done
sort $O/ab.txt
