#!/bin/bash
# K=32 density/tile at 10M vs 900K (lane walk)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python scripts/sweep_tiles.py 10000000 32 3.4,4.2,5.0 4x4x4,4x4x2,8x4x2 0 > gpurun_out/sweep3_10m_k32.log 2>&1 || { echo SWEEP_FAIL; tail gpurun_out/sweep3_10m_k32.log; exit 1; }
grep -v amdgpu gpurun_out/sweep3_10m_k32.log
timeout -k 10 300 python scripts/sweep_tiles.py 3000000 32 3.4,5.0 4x4x4,4x4x2 0 > gpurun_out/sweep3_3m_k32.log 2>&1 || { echo SWEEP_FAIL; tail gpurun_out/sweep3_3m_k32.log; exit 1; }
grep -v amdgpu gpurun_out/sweep3_3m_k32.log
timeout -k 10 200 python bench.py --n 900000 --k 32 --steps 30 --warmup 5 > gpurun_out/b900k_k32.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
tail -1 gpurun_out/b900k_k32.json | cut -c1-200
