#!/bin/bash
# kernel trace of the world-1 distributed step (steady async) -> per-step timeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
R=$PWD
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dist_r2 -o run -- python3 $R/bench.py --dist --no-check --steps 20 --warmup 3 > $R/gpurun_out/prof_dist_r2.log 2>&1 || { echo PROF_FAIL; tail $R/gpurun_out/prof_dist_r2.log; exit 1; }
cd $R
DB=$(find gpurun_out/prof_dist_r2 -name "*.db" | head -1)
python scripts/prof_timeline.py $DB local_meta 40 || python scripts/prof_timeline.py $DB bbox 40
find gpurun_out/prof_dist_r2 -name "*stats*" | head
