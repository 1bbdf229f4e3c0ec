#!/bin/bash
# Pipelined-step A/B of a compile-time variant (_C_<VAR>, KN_C_VARIANT) against _C: engine
# 200 / 50 and 20 / 5, the world-1 distributed pipeline, K=50; two interleaved passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
VAR=${VAR:?}
O=gpurun_out/r5var_$VAR
mkdir -p $O
: > $O/ab.txt
one() {  # label args...
  local label=$1; shift
  MASTER_PORT=$((29700 + RANDOM % 200)) timeout -k 10 120 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('ms_build'))" >> $O/ab.txt
}
for pass in 1 2; do
for v in base $VAR; do
  if [ $v = base ]; then unset KN_C_VARIANT; else export KN_C_VARIANT=$VAR; fi
  one "$v engine 200/50" --steps 200 --warmup 50
  one "$v engine 20/5" --steps 20 --warmup 5
  one "$v dist 200/50" --dist --steps 200 --warmup 50
  one "$v k50 100/30" --k 50 --steps 100 --warmup 30
done
done
sort $O/ab.txt
