#!/bin/bash
# Round 6: the 20 / 5 cold start -- resident pipeline from graphs (default), eager stages
# (KN_PIPE_EAGER=1), graphs uploaded at instantiation (KN_PIPE_GRAPH_UPLOAD=1); two passes; then the
# K=16 query PMC of the current kernel
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6cold
mkdir -p $O
: > $O/cold.txt
one() {  # label env args...
  local label=$1 envs=$2; shift 2
  env $envs timeout -k 10 120 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('ms_solve'))" >> $O/cold.txt
}
for pass in 1 2; do
  for m in "graph KN_X=0" "eager KN_PIPE_EAGER=1" "upload KN_PIPE_GRAPH_UPLOAD=1"; do
    set -- $m
    one "$1 20/5" "$2" --steps 20 --warmup 5
    one "$1 200/50" "$2" --steps 200 --warmup 50
  done
done
sort $O/cold.txt
bash tools/profile.sh pmc 16 900000 > $O/pmc_k16.txt 2>&1 || { echo "PMC_FAIL"; tail $O/pmc_k16.txt; exit 1; }
grep -E "per wave|/ WAVE|conflict|vgpr" $O/pmc_k16.txt
