#!/bin/bash
# Engine with three grid sets (default now) vs two (KN_PIPE_SETS=2): GPU tests + A/B
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5sets3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/ab.txt
one() {  # label env -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 150 python bench.py "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); c=d.get('check',{}); print('$label', round(d['ms_per_step'],4), c.get('bad_rows'), c.get('timed_rows_equal_eager'))" >> $O/ab.txt
}
for pass in 1 2; do
for S in 3 2; do
  one "sets$S 20/5" KN_PIPE_SETS=$S -- --steps 20 --warmup 5
  one "sets$S 200/50" KN_PIPE_SETS=$S -- --steps 200 --warmup 50
  one "sets$S k50 100/30" KN_PIPE_SETS=$S -- --k 50 --steps 100 --warmup 30
  one "sets$S clustered" KN_PIPE_SETS=$S -- --gen clustered --steps 60 --warmup 20
  one "sets$S stream4" KN_PIPE_SETS=$S -- --steps 100 --warmup 20 --stream-clouds 4
done
done
sort $O/ab.txt
