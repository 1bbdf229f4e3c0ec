#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
R=$PWD
for c in "uniform 40000 16" "clustered 900000 16" "uniform 900000 16" "surface 900000 16" "clustered 900000 50" "uniform 900000 50"; do
  timeout -k 10 120 python scripts/diag_tree.py $c >> gpurun_out/diag_tree.jsonl 2>gpurun_out/diag_tree.err || { echo DIAG_FAIL $c; tail gpurun_out/diag_tree.err; exit 1; }
done
cat gpurun_out/diag_tree.jsonl
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_tree -o run -- python3 $R/scripts/diag_tree.py clustered 900000 16 > $R/gpurun_out/prof_tree.log 2>&1 || { echo PROF_FAIL; tail $R/gpurun_out/prof_tree.log; exit 1; }
cd $R && python scripts/kernel_stats.py $(find gpurun_out/prof_tree -name "*.db" | head -1) 14
timeout -k 10 400 python -u -m pytest tests/test_gpu_tree.py -v --timeout 120 --timeout-method thread > gpurun_out/pytest_tree.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/pytest_tree.log | tail -30
exit $rc
