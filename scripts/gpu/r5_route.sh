#!/bin/bash
# routing block size variants (KN_ROUTE_ITEMS: _C_r4k 4096, _C_r16k 16384) vs 1024: world-1 dist
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5route
mkdir -p $O
: > $O/ab.txt
one() {  # label args
  local label=$1; shift
  MASTER_PORT=$((29700 + RANDOM % 200)) timeout -k 10 150 python bench.py "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); c=d.get('check',{}); print('$label', round(d['ms_per_step'],4), c.get('bad_rows_all_ranks'), d.get('ms_route'))" >> $O/ab.txt
}
for pass in 1 2; do
for v in base r4k r16k; do
  if [ $v = base ]; then unset KN_C_VARIANT; else export KN_C_VARIANT=$v; fi
  one "$v dist 200/50" --dist --steps 200 --warmup 50
  one "$v dist 20/5" --dist --steps 20 --warmup 5
done
done
sort $O/ab.txt
