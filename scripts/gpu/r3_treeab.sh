#!/bin/bash
# Round 3: depth-first tree query with stacked per-lane distances (_C) vs round-3 start (_C_dfs0), then the tree GPU tests.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/treeab
mkdir -p $O
timeout -k 10 300 python scripts/ab_tree.py dfs0 900000 16,50 clustered,surface,uniform 6 > $O/ab.jsonl 2> $O/err.log || { echo AB_FAIL; tail -20 $O/err.log; cat $O/ab.jsonl; exit 1; }
cat $O/ab.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
