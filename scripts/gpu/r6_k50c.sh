#!/bin/bash
# Round 6: K=50 walk unroll 2 + re-rank groups of 8 (_C_k50c) vs defaults: query A/B, then
# pipelined K=50 / K=32 bench steps, one module per process, interleaved passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6k50c
mkdir -p $O
: > $O/ab.txt
for k in 50 32; do
  echo "== k50c k=$k" >> $O/ab.txt
  timeout -k 10 200 python scripts/ab_variant.py k50c 900000 $k 14 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $k"; exit 1; }
done
one() {  # label variant args...
  local label=$1 var=$2; shift 2
  if [ -n "$var" ]; then export KN_C_VARIANT=$var; else unset KN_C_VARIANT; fi
  timeout -k 10 120 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('ms_solve'))" >> $O/ab.txt
}
for pass in 1 2; do
  for v in base k50c; do
    vv=$([ $v = base ] && echo "" || echo $v)
    one "$v k50 100/30" "$vv" --k 50 --steps 100 --warmup 30
    one "$v k50 20/5" "$vv" --k 50 --steps 20 --warmup 5
    one "$v k32 100/30" "$vv" --k 32 --steps 100 --warmup 30
  done
done
cat $O/ab.txt
