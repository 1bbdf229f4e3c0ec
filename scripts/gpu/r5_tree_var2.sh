#!/bin/bash
# Tree K=24 / K=32 occupancy variants (_C_<VAR>) against _C; clustered + surfaces, two passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5treevar2
mkdir -p $O
: > $O/ab.txt
one() {  # label args...
  local label=$1; shift
  timeout -k 10 150 python bench.py "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); c=d.get('check',{}); print('$label', round(d['ms_per_step'],4), d.get('exact_path_queries'), c.get('bad_rows'), c.get('bad_id_rows'))" >> $O/ab.txt
}
for pass in 1 2; do
for v in base $VARS; do
  if [ $v = base ]; then unset KN_C_VARIANT; else export KN_C_VARIANT=$v; fi
  one "$v uniform k64" --n 900000 --k 64 --steps 60 --warmup 20
  one "$v clustered k64" --gen clustered --n 900000 --k 64 --steps 20 --warmup 10
  one "$v surface k64" --gen surface --n 900000 --k 64 --steps 20 --warmup 10
done
done
sort $O/ab.txt
