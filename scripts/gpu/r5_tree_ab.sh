#!/bin/bash
# Tree-path A/B of a compile-time variant (_C_<VAR>) against _C: 900K clustered / surfaces, K=16 and
# clustered K=50, pipelined steps, two interleaved passes; then the tree GPU tests on _C
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
VAR=${VAR:?}
O=gpurun_out/r5tree_$VAR
mkdir -p $O
: > $O/ab.txt
one() {  # label args...
  local label=$1; shift
  timeout -k 10 150 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('exact_path_queries'))" >> $O/ab.txt
}
for pass in 1 2; do
for v in base $VAR; do
  if [ $v = base ]; then unset KN_C_VARIANT; else export KN_C_VARIANT=$VAR; fi
  one "$v clustered k16" --gen clustered --n 900000 --k 16 --steps 100 --warmup 20
  one "$v surface k16" --gen surface --n 900000 --k 16 --steps 100 --warmup 20
  one "$v clustered k50" --gen clustered --n 900000 --k 50 --steps 30 --warmup 10
done
done
sort $O/ab.txt
unset KN_C_VARIANT
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
