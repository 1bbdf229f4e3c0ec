#!/bin/bash
# Round 6: serial build of small clouds, bucket totals + prefetch (base) vs the round-5 table + scan
# (old) vs bucket totals without prefetch (pf0); k=8 and k=16
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6small
mkdir -p $O
: > $O/ab.txt
for pass in 1 2; do
  for v in base old pf0; do
    if [ $v = base ]; then unset KN_C_VARIANT; else export KN_C_VARIANT=$v; fi
    for n in 20626 100000 300000; do
      r=$(timeout -k 10 120 python scripts/prof_build.py $n 8 25 2>/dev/null | grep ms_build) || { echo "FAIL $v $n"; exit 1; }
      echo "$v n=$n k=8 ${r##*median}" >> $O/ab.txt
    done
  done
done
unset KN_C_VARIANT
for v in base old; do
  if [ $v = base ]; then unset KN_C_VARIANT; else export KN_C_VARIANT=$v; fi
  timeout -k 10 120 python bench.py --no-check --xyz data/pts20K.xyz --k 8 --steps 200 --warmup 50 > $O/line.json 2> $O/err.txt || { echo "FAIL bench $v"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$v pts20K bench', round(d['ms_per_step'],4), d.get('ms_build'), d.get('ms_solve'))" >> $O/ab.txt
done
cat $O/ab.txt
