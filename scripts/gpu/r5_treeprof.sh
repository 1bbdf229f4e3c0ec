#!/bin/bash
# Kernel stats + last-step timeline of the tree path (900K clustered / surfaces, K=16)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5treeprof
mkdir -p $O
for gen in clustered surface; do
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/$gen -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --gen $gen --n 900000 --k 16 --steps 40 --warmup 10 > $GRAFT_REPO_ROOT/$O/$gen.log 2>&1) || { echo PROF_FAIL; tail $O/$gen.log; exit 1; }
echo "== $gen"; tail -1 $O/$gen.log | cut -c1-150
python scripts/prof_db.py $O/$gen/run_results.db --timeline 40 > $O/$gen.txt
head -20 $O/$gen.txt; tail -41 $O/$gen.txt
done
