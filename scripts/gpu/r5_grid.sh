#!/bin/bash
# Joint A/B: grid sets (KN_PIPE_SETS) x points per binning block (KN_BIN_ITEMS), 256-thread binning
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5grid
mkdir -p $O
: > $O/ab.txt
one() {  # label env -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 150 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4))" >> $O/ab.txt
}
for pass in 1 2; do
for S in 2 3; do
for I in 4096 8192 16384; do
  one "s$S i$I 200/50" KN_PIPE_SETS=$S KN_BIN_ITEMS=$I -- --steps 200 --warmup 50
  one "s$S i$I 20/5" KN_PIPE_SETS=$S KN_BIN_ITEMS=$I -- --steps 20 --warmup 5
  one "s$S i$I k50" KN_PIPE_SETS=$S KN_BIN_ITEMS=$I -- --k 50 --steps 100 --warmup 30
  one "s$S i$I clustered" KN_PIPE_SETS=$S KN_BIN_ITEMS=$I -- --gen clustered --steps 60 --warmup 20
done
done
done
sort $O/ab.txt
