#!/bin/bash
# Second query stream at the default priority (KN_PIPE_AUXPRIO=1) vs the least (shipped), at
# the driver's 20 / 5, 200 / 50, K=50, clustered; two interleaved passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5prio2
mkdir -p $O
: > $O/ab.txt
one() {  # label args...
  local label=$1; shift
  timeout -k 10 120 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4))" >> $O/ab.txt
}
for pass in 1 2 3; do
for ap in 0 1; do
  KN_PIPE_AUXPRIO=$ap one "aux$ap 20/5" --steps 20 --warmup 5
  KN_PIPE_AUXPRIO=$ap one "aux$ap 200/50" --steps 200 --warmup 50
  KN_PIPE_AUXPRIO=$ap KN_PIPE_PRIO=1 one "aux$ap prio1 200/50" --steps 200 --warmup 50
  KN_PIPE_AUXPRIO=$ap one "aux$ap k50 100/30" --k 50 --steps 100 --warmup 30
  KN_PIPE_AUXPRIO=$ap one "aux$ap k50 20/5" --k 50 --steps 20 --warmup 5
  KN_PIPE_AUXPRIO=$ap one "aux$ap k32 100/30" --k 32 --steps 100 --warmup 30
  KN_PIPE_AUXPRIO=$ap one "aux$ap clustered" --gen clustered --steps 60 --warmup 20
  KN_PIPE_AUXPRIO=$ap one "aux$ap surface" --gen surface --steps 60 --warmup 20
  KN_PIPE_AUXPRIO=$ap one "aux$ap stream4" --steps 100 --warmup 20 --stream-clouds 4
done
done
sort $O/ab.txt
