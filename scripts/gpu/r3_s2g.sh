#!/bin/bash
# Round 3 (session 2): outer-pack fix check (oracle diag + A/B), then the full GPU suite, smoke and
# the default (pipelined) bench.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2g
mkdir -p $O
timeout -k 10 400 python scripts/diag_opack.py > $O/diag_opack.log 2>&1 || { echo DIAG_FAIL; tail -20 $O/diag_opack.log; exit 1; }
cat $O/diag_opack.log
timeout -k 10 300 python scripts/ab_multi.py opack 900000 8,12,16,24,32,40 uniform 12 > $O/ab_opack.jsonl 2>> $O/err.log || { echo AB_FAIL; tail -20 $O/err.log; exit 1; }
timeout -k 10 300 python scripts/ab_multi.py opack 900000 16 blue,clustered 8 >> $O/ab_opack.jsonl 2>> $O/err.log || { echo AB2_FAIL; tail -20 $O/err.log; exit 1; }
timeout -k 10 300 python scripts/ab_multi.py opack 300000 16 uniform 12 >> $O/ab_opack.jsonl 2>> $O/err.log || { echo AB3_FAIL; tail -20 $O/err.log; exit 1; }
cat $O/ab_opack.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
cat $O/bench.json
