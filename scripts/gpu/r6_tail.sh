#!/bin/bash
# Round 6: K=50 rows 4 positions per store + a 2-position tail (KN_VEC_TAIL) vs 2 per store
# (_C_notail): GPU grid / tree tests, query A/B, tree A/B, bench steps
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6tail
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py tests/test_gpu_tree.py > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
: > $O/ab.txt
echo "== notail k=50" >> $O/ab.txt
timeout -k 10 200 python scripts/ab_variant.py notail 900000 50 14 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL"; exit 1; }
echo "== tree notail k=50" >> $O/ab.txt
AB_K=50 timeout -k 10 400 python scripts/ab_tree.py _notail 3 30 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "ABT_FAIL"; exit 1; }
one() {  # label variant args...
  local label=$1 var=$2; shift 2
  if [ -n "$var" ]; then export KN_C_VARIANT=$var; else unset KN_C_VARIANT; fi
  timeout -k 10 120 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('ms_build'), d.get('ms_solve'))" >> $O/ab.txt
}
for pass in 1 2; do
  for v in base notail; do
    vv=$([ $v = base ] && echo "" || echo $v)
    one "$v k50 100/30" "$vv" --k 50 --steps 100 --warmup 30
    one "$v k50 20/5" "$vv" --k 50 --steps 20 --warmup 5
  done
done
cat $O/ab.txt
