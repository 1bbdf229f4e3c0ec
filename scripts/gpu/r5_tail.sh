#!/bin/bash
# distributed tail mode (exact finish + flag on the pipeline's tail stream, default) vs off
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5tail
mkdir -p $O
MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 WORLD_SIZE=1 timeout -k 10 400 python -u scripts/diag_dist_pipe.py 30 200000 > $O/diag.log 2>&1 || { echo DIAG_FAIL; tail -30 $O/diag.log; exit 1; }
grep -E "ALL OK|FAIL" $O/diag.log | tail -2
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/ab.txt
one() {  # label env -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" MASTER_PORT=$((29700 + RANDOM % 200)) timeout -k 10 150 python bench.py "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); c=d.get('check',{}); print('$label', round(d['ms_per_step'],4), c.get('bad_rows_all_ranks'), c.get('bad_rows'))" >> $O/ab.txt
}
for pass in 1 2; do
for T in 1 0; do
  one "tail$T 200/50" KN_DIST_TAIL=$T -- --dist --steps 200 --warmup 50
  one "tail$T 20/5" KN_DIST_TAIL=$T -- --dist --steps 20 --warmup 5
  one "tail$T k50" KN_DIST_TAIL=$T -- --dist --k 50 --steps 60 --warmup 20
  one "tail$T clustered" KN_DIST_TAIL=$T -- --dist --gen clustered --steps 40 --warmup 10
done
done
sort $O/ab.txt
