#!/bin/bash
# Round 3 (session 2): kernel stats of the distributed step at world 1 vs the native serial step.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2l
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/pdist -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --steps 30 --warmup 5 > $GRAFT_REPO_ROOT/$O/pdist.log 2>&1) || { echo PROF_FAIL; tail $O/pdist.log; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/pser -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-pipeline --no-check --steps 30 --warmup 5 > $GRAFT_REPO_ROOT/$O/pser.log 2>&1) || { echo PROF_FAIL2; exit 1; }
find $O -name "*kernel_stats.csv" | head
echo done
