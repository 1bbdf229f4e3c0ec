#!/bin/bash
# Three grid sets: the build under two concurrent queries is on the critical path; A/B its stream
# priority (KN_PIPE_PRIO=1 greatest) and the binning block size (KN_BIN_THREADS); two passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5sets3b
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
  one "base 200/50" X=1 -- --steps 200 --warmup 50
  one "prio1 200/50" KN_PIPE_PRIO=1 -- --steps 200 --warmup 50
  one "bin256 200/50" KN_BIN_THREADS=256 -- --steps 200 --warmup 50
  one "bin512 200/50" KN_BIN_THREADS=512 -- --steps 200 --warmup 50
  one "prio1 bin256 200/50" KN_PIPE_PRIO=1 KN_BIN_THREADS=256 -- --steps 200 --warmup 50
  one "base 20/5" X=1 -- --steps 20 --warmup 5
  one "prio1 20/5" KN_PIPE_PRIO=1 -- --steps 20 --warmup 5
  one "base k50" X=1 -- --k 50 --steps 100 --warmup 30
  one "prio1 k50" KN_PIPE_PRIO=1 -- --k 50 --steps 100 --warmup 30
done
sort $O/ab.txt
