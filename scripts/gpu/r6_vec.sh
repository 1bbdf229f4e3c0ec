#!/bin/bash
# Round 6: re-rank rows written in order, V positions per global store (KN_VEC_OUT) vs per-entry
# stores (_C_novec): GPU grid tests, query A/B per K bucket (rows must be identical), bench steps
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6vec
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
: > $O/ab.txt
for k in 16 50 32 8 64 20; do
  echo "== novec k=$k" >> $O/ab.txt
  timeout -k 10 200 python scripts/ab_variant.py novec 900000 $k 12 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $k"; exit 1; }
done
one() {  # label variant args...
  local label=$1 var=$2; shift 2
  if [ -n "$var" ]; then export KN_C_VARIANT=$var; else unset KN_C_VARIANT; fi
  timeout -k 10 120 python bench.py "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('ms_build'), d.get('ms_solve'), d.get('check'))" >> $O/ab.txt
}
for pass in 1 2; do
  for v in base novec; do
    vv=$([ $v = base ] && echo "" || echo $v)
    one "$v 20/5" "$vv" --steps 20 --warmup 5
    one "$v 200/50" "$vv" --steps 200 --warmup 50 --no-check
    one "$v k50 100/30" "$vv" --k 50 --steps 100 --warmup 30 --no-check
  done
done
cat $O/ab.txt
