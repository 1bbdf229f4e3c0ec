#!/bin/bash
# Round 3: where a clustered loopback (8 ranks on one GPU) step spends its time.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/loopprof
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --loopback 8 --n 900000 --k 16 --gen clustered --halo-factor 4 --steps 10 --warmup 3 > $O/hf4.json 2>$O/hf4.err || { tail $O/hf4.err; exit 1; }
tail -1 $O/hf4.json | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python3 $R/bench.py --loopback 8 --n 900000 --k 16 --gen clustered --steps 5 --warmup 3 --no-check > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail $R/$O/prof.log; exit 1; }
cd $R
python scripts/kernel_stats.py $(find $O/prof -name '*.db' | head -1) 30 > $O/kstats.txt 2>&1; cat $O/kstats.txt
