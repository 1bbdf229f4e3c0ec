#!/bin/bash
# Round 3 (session 2): bounds-checked runs of the new paths: tree exact kernel (breadth-first
# sweep; every query forced through it with flags=1) and the world-1 distributed graph step.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2r
mkdir -p $O
timeout -k 10 300 python -u scripts/diag_checked_tree.py > $O/checked_tree.txt 2>&1 || { echo TREE_CHECK_FAIL; tail -20 $O/checked_tree.txt; exit 1; }
tail -4 $O/checked_tree.txt
KN_CHECKED=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29563 RANK=0 WORLD_SIZE=1 timeout -k 10 300 python -u scripts/diag_dist_graph.py 60 200000 > $O/checked_dist_graph.txt 2>&1 || { echo DIST_CHECK_FAIL; tail -20 $O/checked_dist_graph.txt; exit 1; }
tail -4 $O/checked_dist_graph.txt
echo done
