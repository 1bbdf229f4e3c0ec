#!/bin/bash
# world-1 distributed pipeline: eager (default) vs captured per-step graphs, two query streams
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5distcap
mkdir -p $O
: > $O/ab.txt
one() {  # label env -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" MASTER_PORT=$((29700 + RANDOM % 200)) timeout -k 10 150 python bench.py "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); c=d.get('check',{}); print('$label', round(d['ms_per_step'],4), d.get('dist_mode'), c.get('bad_rows_all_ranks'), d.get('host_enqueue_ms_per_step'))" >> $O/ab.txt
}
for pass in 1 2; do
  one "eager 200/50" KN_DIST_CAPTURE=0 -- --dist --steps 200 --warmup 50
  one "graph 200/50" KN_DIST_CAPTURE=1 -- --dist --steps 200 --warmup 50
  one "eager 20/5" KN_DIST_CAPTURE=0 -- --dist --steps 20 --warmup 5
  one "graph 20/5" KN_DIST_CAPTURE=1 -- --dist --steps 20 --warmup 5
  one "eager sets2 200/50" KN_DIST_CAPTURE=0 KN_DIST_SETS=2 -- --dist --steps 200 --warmup 50
done
sort $O/ab.txt
