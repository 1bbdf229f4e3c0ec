#!/bin/bash
# Round 4: the driver's 20 / 5 headline with the eager-row check before the warm-up (default) or
# between the warm-up and the timed steps, interleaved; 200 / 50 for reference.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4chk
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
for rep in 1 2 3; do
  for order in before after; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --check-order $order > "$O/b20_${order}_$rep.json" 2> "$O/b20_${order}_$rep.err" || exit 1
  done
done
timeout -k 10 120 python3 bench.py --steps 200 --warmup 50 > "$O/b200.json" 2> "$O/b200.err" || exit 1
for f in "$O"/*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],4), d.get('check'))")"; done
