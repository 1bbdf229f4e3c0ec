#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/r5b
MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 WORLD_SIZE=1 timeout -k 10 400 python -u scripts/diag_dist_pipe.py 30 200000 > gpurun_out/r5b/diag_dist_pipe.log 2>&1 || { echo DIAG_FAIL; tail -30 gpurun_out/r5b/diag_dist_pipe.log; exit 1; }
grep -E "capture|ALL" gpurun_out/r5b/diag_dist_pipe.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py tests/test_capi.py -x -q --timeout 200 --timeout-method thread -k "long_axis or solve_range or stream" > gpurun_out/r5b/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r5b/pytest.log; exit 1; }
tail -2 gpurun_out/r5b/pytest.log
bash scripts/gpu/r5_ab_split.sh
