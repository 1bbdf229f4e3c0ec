#!/bin/bash
# binning block size (points) x threads at 2M and 4M points, K=16; two passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5bin2
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
for T in 256 1024; do
for I in 8192 16384 32768; do
  one "2M T=$T I=$I" KN_BIN_THREADS=$T KN_BIN_ITEMS=$I -- --n 2000000 --steps 100 --warmup 30
  one "4M T=$T I=$I" KN_BIN_THREADS=$T KN_BIN_ITEMS=$I -- --n 4000000 --steps 60 --warmup 20
done
done
done
sort $O/ab.txt
