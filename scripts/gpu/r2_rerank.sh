#!/bin/bash
# Streaming-window re-rank (new _C) vs the round-1 odd-even re-rank (_C_oldrr): GPU tests of
# the query kernels, then in-process A/B at 900K for K=16/32/50/64 with auto and 2-ring plans.
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_rerank.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/pytest_gpu_rerank.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_rerank.log
O=gpurun_out/ab_rerank.log
: > $O
for kh in "16 0" "32 0" "50 0" "50 2" "64 0" "64 2"; do
  set -- $kh
  echo "== k=$1 halo=$2" >> $O
  timeout -k 10 120 python scripts/ab_plan.py oldrr 900000 $1 $2 10 >> $O 2>&1 || { echo AB_FAIL $kh; tail -5 $O; exit 1; }
done
grep -v amdgpu.ids $O
