#!/bin/bash
# K=64 density/halo (lane walk) at 900K and 3M
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python scripts/sweep_tiles.py 900000 64 2.9,3.4,4.0 4x4x4 2,3 > gpurun_out/sweep5_900k_k64.log 2>&1 || { echo SWEEP_FAIL; tail gpurun_out/sweep5_900k_k64.log; exit 1; }
grep -v amdgpu gpurun_out/sweep5_900k_k64.log
timeout -k 10 300 python scripts/sweep_tiles.py 3000000 64 2.9,3.4,4.0 4x4x4 2,3 > gpurun_out/sweep5_3m_k64.log 2>&1 || { echo SWEEP_FAIL; tail gpurun_out/sweep5_3m_k64.log; exit 1; }
grep -v amdgpu gpurun_out/sweep5_3m_k64.log
