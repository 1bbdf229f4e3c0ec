#!/bin/bash
# first GPU session: tests, bench
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu.py -q -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
  rc2=$?
  echo "bench rc=$rc2"
  tail -8 gpurun_out/bench.log
fi
