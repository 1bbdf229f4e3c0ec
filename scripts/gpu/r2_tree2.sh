#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
for c in "clustered 900000 16" "uniform 900000 16" "surface 900000 16" "blue 900000 16"; do
  timeout -k 10 120 python scripts/diag_tree.py $c >> gpurun_out/diag_tree2.jsonl 2>gpurun_out/diag_tree.err || { echo DIAG_FAIL $c; tail gpurun_out/diag_tree.err; exit 1; }
done
cat gpurun_out/diag_tree2.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_tree.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_r2_grid_tree.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_r2_grid_tree.log
exit $rc
