#!/bin/bash
# Tree-path A/B of compile-time variants (space-separated VARS) against _C: 900K clustered /
# surfaces K=16 and clustered K=50, pipelined, two interleaved passes, rows checked
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5treevar
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
  one "$v clustered k16" --gen clustered --n 900000 --k 16 --steps 60 --warmup 20
  one "$v surface k16" --gen surface --n 900000 --k 16 --steps 60 --warmup 20
  one "$v clustered k8" --gen clustered --n 900000 --k 8 --steps 60 --warmup 20
done
done
sort $O/ab.txt
