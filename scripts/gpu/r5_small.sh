#!/bin/bash
# after shrinking the single-block kernels (steady flag, tree scan top) to 256 threads
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5small
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 WORLD_SIZE=1 timeout -k 10 400 python -u scripts/diag_dist_pipe.py 30 200000 > $O/diag.log 2>&1 || { echo DIAG_FAIL; tail -30 $O/diag.log; exit 1; }
grep -E "ALL OK|FAIL" $O/diag.log | tail -2
: > $O/ab.txt
one() {  # label args
  local label=$1; shift
  MASTER_PORT=$((29700 + RANDOM % 200)) timeout -k 10 150 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4))" >> $O/ab.txt
}
for pass in 1 2; do
  one "dist 200/50" --dist --steps 200 --warmup 50
  one "dist 20/5" --dist --steps 20 --warmup 5
  one "clustered" --gen clustered --steps 60 --warmup 20
  one "surface" --gen surface --steps 60 --warmup 20
  one "engine 200/50" --steps 200 --warmup 50
  one "engine 20/5" --steps 20 --warmup 5
  one "engine k50" --k 50 --steps 100 --warmup 30
done
sort $O/ab.txt
