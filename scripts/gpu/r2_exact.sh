#!/bin/bash
# Threshold-compaction exact kernel: GPU tests, A/B vs round-1 kernels (_C_oldrr), clustered bench
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_capi.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_exact.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/pytest_gpu_exact.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_exact.log
O=gpurun_out/ab_exact.log
: > $O
for kh in "16 0" "50 0" "50 2" "64 2"; do
  set -- $kh
  echo "== uniform k=$1 halo=$2" >> $O
  timeout -k 10 120 python scripts/ab_plan.py oldrr 900000 $1 $2 10 >> $O 2>&1 || { echo AB_FAIL $kh; tail -5 $O; exit 1; }
done
echo "== clustered k=16" >> $O
timeout -k 10 300 python scripts/ab_plan.py oldrr 900000 16 0 3 clustered >> $O 2>&1 || { echo AB_FAIL clustered; tail -5 $O; exit 1; }
grep -v amdgpu.ids $O
timeout -k 10 300 python bench.py --gen clustered --steps 5 --warmup 2 > gpurun_out/bench_clustered.json 2> gpurun_out/bench_clustered.err || { echo BENCH_FAIL; tail gpurun_out/bench_clustered.err; exit 1; }
cat gpurun_out/bench_clustered.json
