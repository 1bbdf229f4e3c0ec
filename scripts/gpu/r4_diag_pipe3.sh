#!/bin/bash
# Round 4: isolate the forced-collective refill failure (mode order, arena cache)
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
run() {
  echo "== $*"
  env "$@" MASTER_PORT=$((29600 + RANDOM % 300)) timeout -k 10 200 python3 scripts/diag_dist_pipe.py 30 200000 $MODES 2>&1 | grep -E "refill|ALL OK|FAILED|^force" | tail -4
}
MODES=1,1 run KN_ROUTE_FUSED=1
MODES=0,1 run KN_ROUTE_FUSED=1 KN_ARENA_CACHE=0
MODES=0,1 run KN_ROUTE_FUSED=1 KN_PIPE_UNROLL=0
