#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5heat2
mkdir -p $O
for rep in 1 2 3; do
for m in none graph pipe; do
  if [ $m = none ]; then unset KN_BENCH_PREHEAT; else export KN_BENCH_PREHEAT=60 KN_BENCH_PREHEAT_MODE=$m; fi
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-check > $O/$m.json 2> $O/$m.err || exit 1
  echo "preheat $m: $(python -c "import json;d=json.loads(open('$O/$m.json').read().splitlines()[-1]);print(round(d['ms_per_step'],4))")"
done
done
