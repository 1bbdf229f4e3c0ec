#!/bin/bash
# A/B of the pipeline events' release scope (KN_EVENT_SCOPE 0 / 1 / 2): engine one / two query
# streams and the world-1 distributed pipeline, 900K K=16, 200 / 50, two interleaved passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5evscope
mkdir -p $O
: > $O/ab.txt
one() {  # label args...
  local label=$1; shift
  MASTER_PORT=$((29700 + RANDOM % 200)) timeout -k 10 120 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4))" >> $O/ab.txt
}
for pass in 1 2; do
for sc in 0 1 2; do
  KN_EVENT_SCOPE=$sc one "scope $sc engine qs2 200/50" --steps 200 --warmup 50
  KN_EVENT_SCOPE=$sc KN_PIPE_QSTREAMS=1 one "scope $sc engine qs1 200/50" --steps 200 --warmup 50
  KN_EVENT_SCOPE=$sc one "scope $sc dist 200/50" --dist --steps 200 --warmup 50
  KN_EVENT_SCOPE=$sc one "scope $sc engine qs2 20/5" --steps 20 --warmup 5
done
done
sort $O/ab.txt
