#!/bin/bash
# Round 3 (session 2): tree exact kernel: breadth-first sweep for bounded queries (one dependent round
# per node); GPU suite, tree-path steps, kernel stats.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2q
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
: > $O/tree.txt
for r in 1 2; do for g in clustered surface; do
  timeout -k 10 200 python bench.py --gen $g --steps 100 --warmup 20 > $O/_t.json 2>> $O/err.log || { echo TREE_FAIL; tail $O/err.log; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/_t.json') if l.startswith('{')][-1]); print('$g', round(d['ms_per_step'],4), '%.3e' % d['value'], d['check'])" >> $O/tree.txt
done; done
cat $O/tree.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/p_cl -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gen clustered --steps 20 --warmup 5 --no-check > $GRAFT_REPO_ROOT/$O/p_cl.log 2>&1) || { echo PROF_FAIL; exit 1; }
python scripts/kernel_stats.py $(find $O/p_cl -name '*.db' | head -1) 8 > $O/kstats_cl.txt 2>&1; cat $O/kstats_cl.txt
echo done
