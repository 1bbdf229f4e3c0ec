#!/bin/bash
# eager batch pipeline over three sets + forced-collective binning: stream tests, A/B
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5batch3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_tree.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/ab.txt
one() {  # label env -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" MASTER_PORT=$((29700 + RANDOM % 200)) timeout -k 10 150 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4))" >> $O/ab.txt
}
for pass in 1 2; do
  one "stream4 i-auto" X=1 -- --steps 200 --warmup 50 --stream-clouds 4
  one "stream4 i4096" KN_BIN_ITEMS=4096 -- --steps 200 --warmup 50 --stream-clouds 4
  one "resident 200/50" X=1 -- --steps 200 --warmup 50
  one "forced" X=1 -- --dist --force-collectives --steps 200 --warmup 50
  one "dist" X=1 -- --dist --steps 200 --warmup 50
done
sort $O/ab.txt
