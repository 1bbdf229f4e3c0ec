#!/bin/bash
# Round-5 baseline on this round's boxes: headline bench (driver's 20 / 5 and 200 / 50), a
# kernel-stats profile of the headline step, and the world-1 distributed path.
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${OUT_DIR:-r5base}
mkdir -p $O
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_20.json 2> $O/bench_20.err || { echo BENCH_FAIL; tail $O/bench_20.err; exit 1; }
cat $O/bench_20.json
timeout -k 10 200 python bench.py --steps 200 --warmup 50 --no-check > $O/bench_200.json 2> $O/bench_200.err || { echo BENCH_FAIL; tail $O/bench_200.err; exit 1; }
cat $O/bench_200.json
timeout -k 10 200 python bench.py --dist --steps 200 --warmup 50 --no-check > $O/dist_200.json 2> $O/dist_200.err || { echo DIST_FAIL; tail $O/dist_200.err; exit 1; }
cat $O/dist_200.json
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1) || { echo PROF_FAIL; exit 1; }
echo done
