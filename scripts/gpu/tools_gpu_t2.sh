#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -20; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -m cProfile -s tottime bench.py --dist --no-check --steps 30 --warmup 5 > gpurun_out/cprof_dist.txt 2> gpurun_out/cprof_dist.err || { echo CPROF_FAIL; tail gpurun_out/cprof_dist.err; exit 1; }
head -45 gpurun_out/cprof_dist.txt
