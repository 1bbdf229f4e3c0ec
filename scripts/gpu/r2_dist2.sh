#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_dist2.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/pytest_dist2.log | tail -40
exit $rc
