#!/bin/bash
# distributed pipeline at the driver's 20 / 5: one vs two query streams, interleaved x3
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5dist20
mkdir -p $O
: > $O/ab.txt
run() {  # label env...
  local label=$1; shift
  env "$@" MASTER_PORT=$((29700 + RANDOM % 200)) timeout -k 10 120 python bench.py --dist --no-check --steps 20 --warmup 5 > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('dist_mode'))" >> $O/ab.txt
}
for pass in 1 2 3; do
run "qs2 sets3 20/5" KN_DIST_QSTREAMS=2
run "qs1 20/5" KN_DIST_QSTREAMS=1
run "qs2 sets2 20/5" KN_DIST_QSTREAMS=2 KN_DIST_SETS=2
echo "engine 20/5 $(timeout -k 10 120 python bench.py --no-check --steps 20 --warmup 5 | python -c "import json,sys; print(round(json.loads(sys.stdin.read().strip().splitlines()[-1])['ms_per_step'],4))")" >> $O/ab.txt
done
sort $O/ab.txt
