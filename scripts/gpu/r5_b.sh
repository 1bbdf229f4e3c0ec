#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out/r5b
bash scripts/gpu/r5_ab_split.sh || exit 1
MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 WORLD_SIZE=1 timeout -k 10 400 python -u scripts/diag_dist_pipe.py 30 200000 > gpurun_out/r5b/diag_dist_pipe.log 2>&1 || { echo DIAG_FAIL; tail -30 gpurun_out/r5b/diag_dist_pipe.log; exit 1; }
grep -E "capture|ALL" gpurun_out/r5b/diag_dist_pipe.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py tests/test_capi.py tests/test_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5b/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r5b/pytest.log; exit 1; }
tail -2 gpurun_out/r5b/pytest.log
timeout -k 10 120 python bench.py --steps 200 --warmup 50 --no-check > gpurun_out/r5b/b200.json 2>gpurun_out/r5b/b200.err && cat gpurun_out/r5b/b200.json
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r5b/b20.json 2>gpurun_out/r5b/b20.err && cat gpurun_out/r5b/b20.json
bash scripts/gpu/r5_qs_dbg.sh
