#!/bin/bash
# After the K-dependent exact epilogue: the GPU suite, then checked K=50 / K=64 / K=16 benches.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4epi
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
for k in 50 64 16; do
  timeout -k 10 200 python3 bench.py --k $k --steps 20 --warmup 5 > "$O/b_k$k.json" 2> "$O/b_k$k.err" || exit 1
  timeout -k 10 200 python3 bench.py --k $k --dist --steps 20 --warmup 5 > "$O/bd_k$k.json" 2> "$O/bd_k$k.err" || exit 1
done
for f in "$O"/*.json; do echo "$(basename $f) $(python3 -c "import json; d=json.load(open('$f')); print(round(d['ms_per_step'],4), d.get('check'))")"; done
