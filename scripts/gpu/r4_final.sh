#!/bin/bash
# Round 4, after the tree traversal changes: GPU tests, tree rows of the suite, loopback halo runs.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4final
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
for g in surface clustered; do
  timeout -k 10 200 python3 bench.py --gen $g --n 900000 --k 16 --steps 100 --warmup 20 > "$O/b_$g.json" 2> "$O/b_$g.err" || exit 1
  timeout -k 10 300 python3 bench.py --loopback 8 --n 900000 --gen $g --steps 10 --warmup 3 > "$O/lb_$g.json" 2> "$O/lb_$g.err" || exit 1
done
timeout -k 10 300 python3 bench.py --gen clustered --n 900000 --k 50 --steps 40 --warmup 10 > "$O/b_clustered_k50.json" 2> "$O/b_clustered_k50.err" || exit 1
for f in "$O"/*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],4), d.get('check'), d.get('stats',{}).get('halo_frac_max'))")"; done
