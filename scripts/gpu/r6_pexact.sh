#!/bin/bash
# Round 6: exact finish placement re-check after the row-store change (KN_PIPE_EXACT=0 query
# stream, =1 side-stream epilogue; default: epilogue for 24 < K <= 64)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6pexact
mkdir -p $O
: > $O/ab.txt
one() {  # label env args...
  local label=$1 ev=$2; shift 2
  env $ev timeout -k 10 120 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4))" >> $O/ab.txt
}
for pass in 1 2 3; do
  one "k16 default 200/50" KN_X=0 --steps 200 --warmup 50
  one "k16 exact=1 200/50" KN_PIPE_EXACT=1 --steps 200 --warmup 50
  one "k16 default 20/5" KN_X=0 --steps 20 --warmup 5
  one "k16 exact=1 20/5" KN_PIPE_EXACT=1 --steps 20 --warmup 5
  one "k50 default 100/30" KN_X=0 --k 50 --steps 100 --warmup 30
  one "k50 exact=0 100/30" KN_PIPE_EXACT=0 --k 50 --steps 100 --warmup 30
done
cat $O/ab.txt
