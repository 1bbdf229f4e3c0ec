#!/bin/bash
# small clouds (pts20K-sized): tile shape vs workgroup count (256 CUs)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 200 python scripts/sweep_tiles.py 20626 8 2.5,3.4 4x4x4,4x4x2,4x2x2,2x2x2 0 > gpurun_out/small_k8.log 2>&1 || { echo SWEEP_FAIL; tail gpurun_out/small_k8.log; exit 1; }
grep -v amdgpu gpurun_out/small_k8.log
timeout -k 10 200 python scripts/sweep_tiles.py 300000 16 3.4 4x4x4,4x4x2,4x2x2 0 > gpurun_out/small_300k.log 2>&1 || { echo SWEEP_FAIL; tail gpurun_out/small_300k.log; exit 1; }
grep -v amdgpu gpurun_out/small_300k.log
