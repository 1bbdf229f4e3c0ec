#!/bin/bash
# Round 3 (session 2): tree leaves of 16 points (_C_leaf16) vs 32.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2f
mkdir -p $O
timeout -k 10 400 python scripts/ab_tree.py leaf16 900000 16,50 clustered,surface 6 > $O/ab_leaf16.jsonl 2>> $O/err.log || { echo AB_FAIL; tail -20 $O/err.log; exit 1; }
cat $O/ab_leaf16.jsonl
timeout -k 10 400 python scripts/diag_opack.py > $O/diag_opack.log 2>&1 || { echo DIAG_FAIL; tail -20 $O/diag_opack.log; exit 1; }
cat $O/diag_opack.log
