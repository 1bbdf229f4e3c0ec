#!/bin/bash
# Round 3: per-phase cycle census of the query kernel + the C-API / distributed GPU tests
# touched by the ADVICE fixes.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/phase
mkdir -p $O
timeout -k 10 200 python scripts/phase_census.py 900000 8 16 32 50 64 > $O/census.jsonl 2> $O/census.err || { echo CENSUS_FAIL; tail $O/census.err; exit 1; }
cat $O/census.jsonl
timeout -k 10 500 python -u -m pytest tests/test_capi.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
