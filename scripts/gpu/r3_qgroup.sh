#!/bin/bash
# Round 3: lane groups per query (KN_QGROUP) -- correctness under G=2/4 and timing vs cloud size.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/qgroup
mkdir -p $O
KN_QGROUP=4 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_g4.log 2>&1 || { echo G4_FAIL; tail -30 $O/pytest_g4.log; exit 1; }
tail -1 $O/pytest_g4.log
KN_QGROUP=2 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "oracle or small or forced or rescan or dense or blue or clustered" > $O/pytest_g2.log 2>&1 || { echo G2_FAIL; tail -30 $O/pytest_g2.log; exit 1; }
tail -1 $O/pytest_g2.log
: > $O/diag.jsonl
for g in 1 2 4; do
KN_QGROUP=$g timeout -k 10 300 python -u scripts/diag_small.py >> $O/diag.jsonl 2>$O/diag.err || { tail $O/diag.err; exit 1; }
done
cat $O/diag.jsonl | cut -c1-220
