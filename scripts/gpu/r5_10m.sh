#!/bin/bash
# 10M K=32 and 12.5M K=16: query streams / grid sets A/B, two passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r510m
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
  one "10M qs2 sets3" X=1 -- --n 10000000 --k 32 --steps 20 --warmup 10
  one "10M qs2 sets2" KN_PIPE_SETS=2 -- --n 10000000 --k 32 --steps 20 --warmup 10
  one "10M qs1" KN_PIPE_QSTREAMS=1 -- --n 10000000 --k 32 --steps 20 --warmup 10
  one "12.5M qs2 sets3" X=1 -- --n 12500000 --k 16 --steps 20 --warmup 10
  one "12.5M qs1" KN_PIPE_QSTREAMS=1 -- --n 12500000 --k 16 --steps 20 --warmup 10
done
sort $O/ab.txt
