#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/diag_clustered.py 900000 16 > gpurun_out/diag_clust.log 2>&1 || { echo DIAG_FAIL; tail gpurun_out/diag_clust.log; exit 1; }
grep -v amdgpu.ids gpurun_out/diag_clust.log
R=$PWD
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_clust -o run -- python3 $R/bench.py --gen clustered --no-check --steps 5 --warmup 2 > $R/gpurun_out/prof_clust.log 2>&1 || { echo PROF_FAIL; tail $R/gpurun_out/prof_clust.log; exit 1; }
cd $R && python scripts/kernel_stats.py $(find gpurun_out/prof_clust -name "*.db" | head -1) 8
