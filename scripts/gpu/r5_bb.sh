#!/bin/bash
# KN_BUILD_BATCH=1 (4 points per thread loaded before their LDS atomics, _C_bb1) vs shipped, pipelined
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5bb
mkdir -p $O
: > $O/ab.txt
one() {  # label args
  local label=$1; shift
  MASTER_PORT=$((29700 + RANDOM % 200)) timeout -k 10 150 python bench.py "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); c=d.get('check',{}); print('$label', round(d['ms_per_step'],4), d.get('ms_build'), c.get('bad_rows'), c.get('bad_rows_all_ranks'))" >> $O/ab.txt
}
for pass in 1 2; do
for v in base bb1; do
  if [ $v = base ]; then unset KN_C_VARIANT; else export KN_C_VARIANT=$v; fi
  one "$v 200/50" --steps 200 --warmup 50
  one "$v 20/5" --steps 20 --warmup 5
  one "$v clustered" --gen clustered --steps 60 --warmup 20
  one "$v dist" --dist --steps 200 --warmup 50
done
done
sort $O/ab.txt
