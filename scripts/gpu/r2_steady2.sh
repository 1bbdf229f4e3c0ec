#!/bin/bash
# GPU suite + distributed step (world 1, RCCL) after the gid-carrying scatter and the block-wide
# steady flag + its kernel trace, and the native headline.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/steady2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for i in 1 2; do
  timeout -k 10 120 python bench.py > $O/native_$i.json 2> $O/native_$i.err || { echo FAIL; tail $O/native_$i.err; exit 1; }
  cut -c1-220 $O/native_$i.json
  timeout -k 10 180 python bench.py --dist > $O/dist_$i.json 2> $O/dist_$i.err || { echo DIST_FAIL; tail $O/dist_$i.err; exit 1; }
  cut -c1-220 $O/dist_$i.json; grep -o '"check": {[^}]*}' $O/dist_$i.json
done
timeout -k 10 300 python bench.py --dist --gen clustered > $O/dist_clustered.json 2> $O/dist_clustered.err || { echo DIST_FAIL; tail $O/dist_clustered.err; exit 1; }
cut -c1-220 $O/dist_clustered.json; grep -o '"check": {[^}]*}' $O/dist_clustered.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_dist -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --no-check --steps 20 > $GRAFT_REPO_ROOT/$O/prof_dist.log 2>&1 || { echo PROF_FAIL; tail $GRAFT_REPO_ROOT/$O/prof_dist.log; exit 1; }
echo done
