#!/bin/bash
# build stream at the greatest priority (KN_PIPE_PRIO=1) vs default, mid-size clouds; two passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5prios
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
for P in 0 1; do
  one "prio$P 300K" KN_PIPE_PRIO=$P -- --n 300000 --steps 200 --warmup 50
  one "prio$P 400K" KN_PIPE_PRIO=$P -- --n 400000 --steps 200 --warmup 50
  one "prio$P 350K" KN_PIPE_PRIO=$P -- --n 350000 --steps 200 --warmup 50
  one "prio$P 900K" KN_PIPE_PRIO=$P -- --steps 200 --warmup 50
done
done
sort $O/ab.txt
