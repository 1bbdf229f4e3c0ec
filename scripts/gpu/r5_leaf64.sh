#!/bin/bash
# 64-point leaves (default) vs 32 (_C_lb5): tree GPU tests, distributed/tree tests, A/B incl. K=64
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5leaf64
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/ab.txt
one() {  # label args...
  local label=$1; shift
  timeout -k 10 150 python bench.py "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); c=d.get('check',{}); print('$label', round(d['ms_per_step'],4), d.get('exact_path_queries'), c.get('bad_rows'), c.get('bad_id_rows'))" >> $O/ab.txt
}
for pass in 1 2; do
for v in base lb5; do
  if [ $v = base ]; then unset KN_C_VARIANT; else export KN_C_VARIANT=$v; fi
  one "$v clustered k8" --gen clustered --n 900000 --k 8 --steps 60 --warmup 20
  one "$v clustered k32" --gen clustered --n 900000 --k 32 --steps 30 --warmup 10
  one "$v clustered k64" --gen clustered --n 900000 --k 64 --steps 20 --warmup 10
  one "$v surface k50" --gen surface --n 900000 --k 50 --steps 20 --warmup 10
  one "$v clustered 3M k16" --gen clustered --n 3000000 --k 16 --steps 20 --warmup 10
done
done
sort $O/ab.txt
