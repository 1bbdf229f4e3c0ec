#!/bin/bash
# Round 6: kernel stats of the headline bench (900K K=16) and a dispatch timeline of the world-1
# native distributed step (which kernels / memsets / copies a step enqueues)
set -o pipefail
R=$PWD
O=$R/gpurun_out/r6prof
mkdir -p $O
bash tools/profile.sh kstats --steps 50 --warmup 20 > $O/headline.txt 2>&1 || { echo FAIL headline; tail $O/headline.txt; exit 1; }
export PYTHONPATH=$R TMPDIR=/tmp KN_BENCH_SUPERVISE=0
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dist -o run -- python3 $R/bench.py --no-check --dist --steps 30 --warmup 10 > $O/dist.log 2>&1 || { echo FAIL dist; tail $O/dist.log; exit 1; }
db=$(find $O/dist -name "*.db" | head -1)
python3 $R/scripts/prof_db.py "$db" --timeline 80 > $O/dist_summary.txt
cat $O/headline.txt | head -20; cat $O/dist_summary.txt
