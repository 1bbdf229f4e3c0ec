#!/bin/bash
# K=50 density/halo at 3M (does the 900K choice generalise?), then GPU tests + BASELINE suite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python scripts/sweep_tiles.py 3000000 50 2.9,3.4 4x4x4 2,3 > gpurun_out/sweep4_3m_k50.log 2>&1 || { echo SWEEP_FAIL; tail gpurun_out/sweep4_3m_k50.log; exit 1; }
grep -v amdgpu gpurun_out/sweep4_3m_k50.log
bash scripts/gpu/tools_gpu_t7.sh
