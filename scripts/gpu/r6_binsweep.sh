#!/bin/bash
# Round 6: pipelined binning block shape re-checked after the bucket-totals build (KN_BIN_THREADS,
# KN_BIN_ITEMS; defaults 256 threads, ~16K points per block up to 4M points)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6binsweep
mkdir -p $O
: > $O/ab.txt
one() {  # label env args...
  local label=$1 ev=$2; shift 2
  env $ev timeout -k 10 120 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4))" >> $O/ab.txt
}
for pass in 1 2; do
  for cfg in "default KN_X=0" "t1024 KN_BIN_THREADS=1024" "i8k KN_BIN_ITEMS=8192" "i4k KN_BIN_ITEMS=4096" "t512 KN_BIN_THREADS=512"; do
    set -- $cfg
    one "$1 900K 200/50" $2 --steps 200 --warmup 50
    one "$1 300K 200/50" $2 --n 300000 --steps 200 --warmup 50
  done
done
cat $O/ab.txt
