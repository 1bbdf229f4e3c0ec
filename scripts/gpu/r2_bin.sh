#!/bin/bash
# A/B of the binning block size (KN_BIN_THREADS) + kernel traces of the native and the
# distributed (world 1, RCCL) steps.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/bin
mkdir -p $O
for t in 256 1024 256 1024; do
  KN_BIN_THREADS=$t timeout -k 10 120 python bench.py --no-check > $O/b_$t.json 2> $O/b_$t.err || { echo FAIL $t; tail $O/b_$t.err; exit 1; }
  echo "threads $t $(python -c "import json;d=json.load(open('$O/b_$t.json'));print(d['ms_per_step'], d['ms_build'])")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_native -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --steps 20 > $GRAFT_REPO_ROOT/$O/prof_native.log 2>&1 || { echo PROF_FAIL; tail $GRAFT_REPO_ROOT/$O/prof_native.log; exit 1; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_dist -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --no-check --steps 20 > $GRAFT_REPO_ROOT/$O/prof_dist.log 2>&1 || { echo PROF_FAIL; tail $GRAFT_REPO_ROOT/$O/prof_dist.log; exit 1; }
find $GRAFT_REPO_ROOT/$O -name "*.csv" | head
