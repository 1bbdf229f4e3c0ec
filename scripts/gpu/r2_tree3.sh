#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
for c in "clustered 900000 16" "uniform 900000 16" "surface 900000 16" "clustered 900000 50"; do
  timeout -k 10 120 python scripts/diag_tree.py $c >> gpurun_out/diag_tree3.jsonl 2>gpurun_out/diag_tree.err || { echo DIAG_FAIL $c; tail gpurun_out/diag_tree.err; exit 1; }
done
cat gpurun_out/diag_tree3.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py tests/test_capi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_tree3.log 2>&1
rc=$?
grep -E "FAIL|passed|failed|Error" gpurun_out/pytest_tree3.log | tail -20
[ $rc -eq 0 ] || exit $rc
for g in clustered surface uniform; do
  timeout -k 10 200 python bench.py --gen $g --steps 20 --warmup 3 > gpurun_out/bench_tree_$g.json 2>gpurun_out/bench_tree_$g.err || { echo BENCH_FAIL $g; tail gpurun_out/bench_tree_$g.err; exit 1; }
  cat gpurun_out/bench_tree_$g.json
done
