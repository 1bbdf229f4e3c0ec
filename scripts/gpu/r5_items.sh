#!/bin/bash
# Points per binning block (KN_BIN_ITEMS) with 256-thread blocks, pipelined; two passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5items
mkdir -p $O
: > $O/ab.txt
one() {  # label env -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 150 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('ms_build'))" >> $O/ab.txt
}
for pass in 1 2; do
for I in 1024 2048 4096 8192; do
  one "items$I 200/50" KN_BIN_ITEMS=$I -- --steps 200 --warmup 50
  one "items$I clustered" KN_BIN_ITEMS=$I -- --gen clustered --steps 60 --warmup 20
  one "items$I k32" KN_BIN_ITEMS=$I -- --k 32 --steps 100 --warmup 30
done
done
sort $O/ab.txt
: > $O/ab2.txt
two() {  # label env -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 150 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4))" >> $O/ab2.txt
}
for pass in 1 2; do
for S in 2 3; do
  two "sets$S 200/50" KN_PIPE_SETS=$S -- --steps 200 --warmup 50
  two "sets$S 20/5" KN_PIPE_SETS=$S -- --steps 20 --warmup 5
  two "sets$S k50" KN_PIPE_SETS=$S -- --k 50 --steps 100 --warmup 30
done
done
sort $O/ab2.txt
