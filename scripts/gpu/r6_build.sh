#!/bin/bash
# Round 6: serial build census at 900K (and 300K): event-timed ms_build per prepare, then a kernel
# trace of the same loop split into kernel time and inter-kernel gaps
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp KN_BENCH_SUPERVISE=0
R=$PWD
O=$R/gpurun_out/r6build
mkdir -p $O
timeout -k 10 120 python scripts/prof_build.py 900000 16 20 > $O/plain.txt 2>&1 || { echo FAIL plain; tail $O/plain.txt; exit 1; }
timeout -k 10 120 python scripts/prof_build.py 300000 16 20 >> $O/plain.txt 2>&1 || { echo FAIL plain300; tail $O/plain.txt; exit 1; }
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/trace -o run -- python3 $R/scripts/prof_build.py 900000 16 20 > $O/trace.log 2>&1 || { echo FAIL trace; tail $O/trace.log; exit 1; }
db=$(find $O/trace -name "*.db" | head -1)
python3 $R/scripts/prof_db.py "$db" --timeline 30 > $O/summary.txt
cat $O/plain.txt $O/summary.txt
