#!/bin/bash
# full GPU suite + smoke + benches + K=50 / K=64 rows
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5full4
mkdir -p $O
OUT_DIR=r5full4 bash scripts/gpu/r5_full.sh || exit 1
for k in 50 64; do
timeout -k 10 150 python bench.py --k $k --steps 100 --warmup 30 > $O/k$k.json 2> $O/k$k.err || { echo "K$k FAIL"; tail $O/k$k.err; exit 1; }
python -c "import json; d=json.loads(open('$O/k$k.json').read().strip().splitlines()[-1]); print('k$k', round(d['ms_per_step'],4), d.get('exact_path_queries'), d.get('check'))"
done
