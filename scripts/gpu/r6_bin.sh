#!/bin/bash
# Round 6: bucket offsets by totals atomics (no scan kernel) + point prefetch in the bucketed
# build. Correctness (GPU build/layout tests), then serial ms_build per variant (one module per
# process, interleaved), then pipelined bench steps.
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6bin
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
: > $O/ab.txt
for pass in 1 2 3; do
  for v in base old pf; do
    if [ $v = base ]; then unset KN_C_VARIANT; else export KN_C_VARIANT=$v; fi
    for n in 900000 300000 4000000; do
      r=$(timeout -k 10 120 python scripts/prof_build.py $n 16 25 2>/dev/null | grep ms_build) || { echo "FAIL $v $n"; exit 1; }
      echo "$v n=$n ${r##*median}" >> $O/ab.txt
    done
  done
done
unset KN_C_VARIANT
one() {  # label variant args...
  local label=$1 var=$2; shift 2
  if [ -n "$var" ]; then export KN_C_VARIANT=$var; else unset KN_C_VARIANT; fi
  timeout -k 10 120 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('ms_build'), d.get('ms_solve'))" >> $O/ab.txt
}
for pass in 1 2; do
  for v in base old; do
    vv=$([ $v = base ] && echo "" || echo $v)
    one "$v 200/50" "$vv" --steps 200 --warmup 50
    one "$v 20/5" "$vv" --steps 20 --warmup 5
    one "$v 300K" "$vv" --n 300000 --steps 200 --warmup 50
  done
done
cat $O/ab.txt
