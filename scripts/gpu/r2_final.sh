#!/bin/bash
# Final consolidated measurement in ONE box: native vs distributed (world 1, RCCL) alternating,
# K=50/64, clustered; smoke.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/final
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
run() { local name=$1; shift; timeout -k 10 240 python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);print('$name', round(d['ms_per_step'],4), '%.3e' % d['value'], d.get('ms_build'), d.get('exact_path_queries'), d['check'])"; }
for i in 1 2 3; do run native_$i; run dist_$i --dist; done
run k50 --k 50
run k64 --k 64
run clustered --gen clustered
run strong_dist --dist --scaling strong
echo done
