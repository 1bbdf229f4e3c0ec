#!/bin/bash
# stream of distinct clouds: eager batch pipeline (default) vs captured batch graphs; tests of both
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5batch
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py -x -q --timeout 120 --timeout-method thread -k "stream" > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
KN_BATCH_MODE=graph timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py -x -q --timeout 120 --timeout-method thread -k "stream" > $O/pytest_graph.log 2>&1 || { echo TESTS_FAIL_GRAPH; tail -30 $O/pytest_graph.log; exit 1; }
tail -1 $O/pytest_graph.log
: > $O/ab.txt
one() {  # label args...
  local label=$1; shift
  timeout -k 10 120 python bench.py "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('check'))" >> $O/ab.txt
}
for pass in 1 2; do
  one "eager stream4 200/50" --steps 200 --warmup 50 --stream-clouds 4
  KN_BATCH_MODE=graph one "graph stream4 200/50" --steps 200 --warmup 50 --stream-clouds 4
  one "eager stream4 k50 100/30" --k 50 --steps 100 --warmup 30 --stream-clouds 4
  KN_BATCH_MODE=graph one "graph stream4 k50 100/30" --k 50 --steps 100 --warmup 30 --stream-clouds 4
  one "resident 200/50" --steps 200 --warmup 50 --no-check
  one "resident k50 100/30" --k 50 --steps 100 --warmup 30 --no-check
done
sort $O/ab.txt
