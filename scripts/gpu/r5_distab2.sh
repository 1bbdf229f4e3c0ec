#!/bin/bash
# world-1 distributed pipeline A/B with the second query stream at the default priority
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5distab2
mkdir -p $O
: > $O/ab.txt
run() {  # label env...
  local label=$1; shift
  env "$@" MASTER_PORT=$((29700 + RANDOM % 200)) timeout -k 10 120 python bench.py --dist --no-check --steps 200 --warmup 50 > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('dist_mode'))" >> $O/ab.txt
}
for pass in 1 2; do
run "qs1" KN_DIST_QSTREAMS=1
run "qs2 sets2 defer0" KN_DIST_QSTREAMS=2 KN_DIST_SETS=2 KN_DIST_DEFER=0
run "qs2 sets2 defer1" KN_DIST_QSTREAMS=2 KN_DIST_SETS=2
run "qs2 sets3 defer1" KN_DIST_QSTREAMS=2 KN_DIST_SETS=3
run "qs2 sets3 defer0" KN_DIST_QSTREAMS=2 KN_DIST_SETS=3 KN_DIST_DEFER=0
run "qs2 sets2 defer0 auxlow" KN_DIST_QSTREAMS=2 KN_DIST_SETS=2 KN_DIST_DEFER=0 KN_PIPE_AUXPRIO=0
done
sort $O/ab.txt
