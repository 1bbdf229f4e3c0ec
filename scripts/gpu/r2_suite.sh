#!/bin/bash
# Round-2 measurement suite for DESIGN §6: headline, K sweep, distributions, 10M K=32, loopback
# 8 x 900K and 8 x 12.5M (100M), strong scaling rehearsal (loopback 8 x 112.5K).
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/suite
mkdir -p $O
run() { # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  python - "$name" "$O/$name.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[1], round(d["ms_per_step"], 4), "ms", f'{d["value"]:.3e} q/s', d.get("ms_build"), d.get("exact_path_queries"), d.get("check"), d.get("stats", ""))
PY
}
run k16 120 --steps 50
run k8 120 --k 8
run k32 120 --k 32
run k50 120 --k 50
run k64 120 --k 64
run blue_k16 120 --gen blue
run clustered_k16 120 --gen clustered
run surface_k16 120 --gen surface
run pts20k_k8 120 --xyz data/pts20K.xyz --k 8
run 10m_k32 300 --n 10000000 --k 32 --steps 10 --warmup 2
run dist_w1 180 --dist
run loop8_900k 600 --loopback 8 --steps 10 --warmup 3
run loop8_clustered 600 --loopback 8 --gen clustered --steps 5 --warmup 2
run loop8_100m 900 --loopback 8 --n 12500000 --steps 3 --warmup 1 --no-check
echo done
