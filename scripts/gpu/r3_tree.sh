#!/bin/bash
# Round 3: sort-free, graph-capturable tree path: tree tests, grid-vs-tree diagnostics, clustered /
# surface bench (the tree step now replays from the hipGraph), kernel table of the clustered step.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/tree
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for g in clustered surface uniform; do
  timeout -k 10 120 python scripts/diag_tree.py $g 900000 16 >> $O/diag.jsonl 2>> $O/err.log || { echo DIAG_FAIL; tail $O/err.log; exit 1; }
done
cat $O/diag.jsonl
timeout -k 10 200 python bench.py --gen clustered --steps 20 --warmup 3 > $O/bench_clustered.json 2>> $O/err.log || { echo BENCH_FAIL; tail $O/err.log; exit 1; }
cat $O/bench_clustered.json
timeout -k 10 200 python bench.py --gen surface --steps 20 --warmup 3 > $O/bench_surface.json 2>> $O/err.log || { echo BENCH_FAIL; tail $O/err.log; exit 1; }
cat $O/bench_surface.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gen clustered --no-check --steps 10 --warmup 2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo PROF_FAIL; tail $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo done
