#!/bin/bash
# Cold-start structure of the pipelined headline: 20 timed steps after W warm-up steps, and after
# 60 warm-up steps + an idle gap (KN_BENCH_GAP_MS); two interleaved passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5warm
mkdir -p $O
: > $O/ab.txt
one() {  # label args...
  local label=$1; shift
  timeout -k 10 120 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4))" >> $O/ab.txt
}
for pass in 1 2; do
for w in 5 15 30 45 60 100; do one "W=$w K=20" --steps 20 --warmup $w; done
KN_BENCH_GAP_MS=50 one "W=60 gap50ms K=20" --steps 20 --warmup 60
KN_BENCH_GAP_MS=500 one "W=60 gap500ms K=20" --steps 20 --warmup 60
one "W=5 K=100" --steps 100 --warmup 5
one "W=5 K=200" --steps 200 --warmup 5
done
cat $O/ab.txt
