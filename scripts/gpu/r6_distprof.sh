#!/bin/bash
# Round 6 end: world-1 native distributed step timeline after the fused step check and the
# route_count-zeroed bucket totals
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6distprof
mkdir -p $O
export PYTHONPATH=$R TMPDIR=/tmp KN_BENCH_SUPERVISE=0
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dist -o run -- python3 $R/bench.py --no-check --dist --steps 30 --warmup 10 > $O/dist.log 2>&1 || { echo FAIL dist; tail $O/dist.log; exit 1; }
db=$(find $O/dist -name "*.db" | head -1)
python3 $R/scripts/prof_db.py "$db" --timeline 40 > $O/summary.txt
cat $O/summary.txt
