#!/bin/bash
# GPU box: distributed-path tests + world-1 dist bench (both layouts) + tile-kernel work stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_dist.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu_dist.log; exit 1; }
echo PYTEST_OK
for L in partitioned scattered; do
  timeout -k 10 240 python bench.py --dist --layout $L --steps 20 --warmup 5 > gpurun_out/bench_dist_$L.json 2> gpurun_out/bench_dist_$L.err || { echo BENCHD_FAIL; tail gpurun_out/bench_dist_$L.err; exit 1; }
  cat gpurun_out/bench_dist_$L.json
done
timeout -k 10 120 python scripts/diag_work.py 900000 16 > gpurun_out/diag_work.json 2>&1 || { echo DIAG_FAIL; tail gpurun_out/diag_work.json; exit 1; }
cat gpurun_out/diag_work.json
