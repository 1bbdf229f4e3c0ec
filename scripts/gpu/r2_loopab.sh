#!/bin/bash
# A/B of the loopback 8 x 900K step: this tree vs the previous commit (built in .ab_old).
set -o pipefail
O=$PWD/gpurun_out/loopab
mkdir -p $O
for i in 1 2 3; do
  for v in new old; do
    if [ $v = new ]; then D=$PWD; else D=$PWD/.ab_old; fi
    (cd $D && PYTHONPATH=$D timeout -k 10 300 python bench.py --loopback 8 --steps 10 --warmup 3 --no-check > $O/${v}_$i.json 2> $O/${v}_$i.err) || { echo FAIL $v; tail $O/${v}_$i.err; exit 1; }
    echo "$v $i $(python -c "import json;print(round(json.load(open('$O/${v}_$i.json'))['ms_per_step'],3))")"
  done
done
for v in new old; do
  if [ $v = new ]; then D=$PWD; else D=$PWD/.ab_old; fi
  (cd $D && PYTHONPATH=$D timeout -k 10 300 python bench.py --loopback 8 --steps 10 --warmup 3 --no-check --sync-steps > $O/${v}_sync.json 2> $O/${v}_sync.err) || { echo FAIL $v; exit 1; }
  echo "$v sync $(python -c "import json;print(round(json.load(open('$O/${v}_sync.json'))['ms_per_step'],3))")"
done
