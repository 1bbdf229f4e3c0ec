#!/bin/bash
# Round 3: collect-then-select lane walk (_C) vs the round-2 lane walk (_C_old): identical rows,
# exact-path counters and query time at 900K over K and clouds; then the GPU test suite.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/collect
mkdir -p $O
timeout -k 10 300 python scripts/ab_multi.py old 900000 8,16,32,50,64 uniform,blue 10 > $O/ab.jsonl 2> $O/ab.err || { echo AB_FAIL; tail -20 $O/ab.err; cat $O/ab.jsonl; exit 1; }
cat $O/ab.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
