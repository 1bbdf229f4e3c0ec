#!/bin/bash
# K=50 / K=64 A/B: exact finish on the query stream vs epilogue (KN_PIPE_EXACT), two margin slots
# (_C_m2) vs one; pipelined 100 / 30, two passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5k50
mkdir -p $O
: > $O/ab.txt
one() {  # label args...
  local label=$1; shift
  timeout -k 10 150 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('exact_path_queries'))" >> $O/ab.txt
}
for pass in 1 2; do
for k in 50 64; do
  one "k$k base" --k $k --steps 100 --warmup 30
  KN_PIPE_EXACT=0 one "k$k exact-on-query-stream" --k $k --steps 100 --warmup 30
  KN_C_VARIANT=m2 one "k$k margin2" --k $k --steps 100 --warmup 30
  KN_C_VARIANT=m2 KN_PIPE_EXACT=0 one "k$k margin2 exact-on-query-stream" --k $k --steps 100 --warmup 30
done
  one "k32 base" --k 32 --steps 100 --warmup 30
  KN_PIPE_EXACT=1 one "k32 exact-epilogue" --k 32 --steps 100 --warmup 30
  one "k16 base" --k 16 --steps 200 --warmup 50
  KN_PIPE_EXACT=1 one "k16 exact-epilogue" --k 16 --steps 200 --warmup 50
done
sort $O/ab.txt
