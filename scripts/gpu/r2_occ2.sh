#!/bin/bash
# Occupancy plan sweep after moving the cooperative re-scan buffer into the staged area's tail
# (LDS per workgroup 39.5 -> 35.4 KB at the default plan); density x capacity slack.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/occ2
mkdir -p $O
timeout -k 10 300 python scripts/sweep_occ.py 900000 16 3.43,3.2,3.0,2.8 5,3,2,1.5 > $O/k16.txt 2>&1 || { echo FAIL; tail $O/k16.txt; exit 1; }
cat $O/k16.txt
timeout -k 10 300 python scripts/sweep_occ.py 3000000 16 3.43,3.0 5,2 > $O/k16_3m.txt 2>&1 || { echo FAIL; tail $O/k16_3m.txt; exit 1; }
cat $O/k16_3m.txt
timeout -k 10 200 python bench.py --no-check > $O/bench.json 2>&1 || { echo FAIL; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench.json
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
