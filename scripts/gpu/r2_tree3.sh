#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py tests/test_capi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_tree3.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/pytest_tree3.log | tail -40
[ $rc -eq 0 ] || exit $rc
for g in clustered surface uniform; do
  timeout -k 10 200 python bench.py --gen $g --steps 20 --warmup 3 > gpurun_out/bench_tree_$g.json 2>gpurun_out/bench_tree_$g.err || { echo BENCH_FAIL $g; tail gpurun_out/bench_tree_$g.err; exit 1; }
  cat gpurun_out/bench_tree_$g.json
done
timeout -k 10 200 python bench.py --gen clustered --k 50 --steps 10 --warmup 2 > gpurun_out/bench_tree_clustered50.json 2>gpurun_out/bench_tree_c50.err || { echo BENCH_FAIL c50; tail gpurun_out/bench_tree_c50.err; exit 1; }
cat gpurun_out/bench_tree_clustered50.json
