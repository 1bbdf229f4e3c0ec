#!/bin/bash
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 5 180 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1; echo rc=$?; tail -1 gpurun_out/bench.log | cut -c1-200; grep "eager done" gpurun_out/bench.log
[ -s gpurun_out/bench.log ] || exit 1
PYTHONPATH=. timeout -k 5 600 python -m pytest tests/test_gpu.py -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; echo rc=$?; tail -4 gpurun_out/pytest_gpu.log
KN_CHECKED=1 PYTHONPATH=. timeout -k 5 180 python -c "
import torch, cuda_knearests_amd as kn
from cuda_knearests_amd.utils import uniform_cloud
p = uniform_cloud(900000, 0, device='cuda')
g = kn.build_grid(p, 16); i, d, info = kn.query(g, 16, return_info=True); print('checked counters', info['counters'].tolist())
from cuda_knearests_amd._ext import load; print('debug', load().debug_words(False))
"
