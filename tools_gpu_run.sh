#!/bin/bash
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 5 180 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1; echo rc=$?; tail -1 gpurun_out/bench.log | cut -c1-250; grep "eager done" gpurun_out/bench.log
[ -s gpurun_out/bench.log ] || exit 1
PYTHONPATH=. timeout -k 5 600 python -m pytest tests/test_gpu.py -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; echo rc=$?; tail -4 gpurun_out/pytest_gpu.log
