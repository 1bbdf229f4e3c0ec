#!/bin/bash
# GPU box run: gpu tests, 1-GPU bench (native + distributed path at world 1), rocprofv3 kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
echo PYTEST_OK
timeout -k 10 240 python bench.py --steps 50 --warmup 10 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAIL; tail gpurun_out/bench.err; exit 1; }
echo BENCH_OK; cat gpurun_out/bench.json
timeout -k 10 240 python bench.py --dist --steps 20 --warmup 5 > gpurun_out/bench_dist1.json 2> gpurun_out/bench_dist1.err || { echo BENCHD_FAIL; tail gpurun_out/bench_dist1.err; exit 1; }
echo BENCHD_OK; cat gpurun_out/bench_dist1.json
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dist -o run -- python3 $R/bench.py --dist --no-check --steps 10 --warmup 3 > $R/gpurun_out/prof_dist.log 2>&1 || { echo PROF_FAIL; tail $R/gpurun_out/prof_dist.log; exit 1; }
echo PROF_OK
