#!/bin/bash
# Round 6: the distributed build's bucket totals zeroed by route_count (no memset node):
# distributed GPU tests + diag, then world-1 steps
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6dfill
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_distributed.py > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 300 python scripts/diag_dist_pipe.py > $O/diag.txt 2>&1 || { echo DIAG_FAIL; tail -30 $O/diag.txt; exit 1; }
tail -1 $O/diag.txt
: > $O/ab.txt
for pass in 1 2 3; do
  timeout -k 10 150 python bench.py --no-check --dist --steps 200 --warmup 50 > $O/line.json 2> $O/err.txt || { echo "FAIL"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('dist 200/50', round(d['ms_per_step'],4))" >> $O/ab.txt
  timeout -k 10 150 python bench.py --no-check --steps 200 --warmup 50 > $O/line.json 2> $O/err.txt || { echo "FAIL"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('engine 200/50', round(d['ms_per_step'],4))" >> $O/ab.txt
done
cat $O/ab.txt
