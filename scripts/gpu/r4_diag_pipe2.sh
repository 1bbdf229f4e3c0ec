#!/bin/bash
# Round 4: the world-1 RCCL pipeline diagnostics with the fused and the three-kernel router
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
for fused in 1; do
  echo "== fused $fused"
  MASTER_PORT=$((29600 + RANDOM % 300)) KN_DIAG_VERBOSE=1 KN_ROUTE_FUSED=$fused timeout -k 10 200 python3 scripts/diag_dist_pipe.py 30 200000 2>&1 | grep -v "NCCL WARN\|RCCL\|version\|Hostname\|Librccl" | tail -12
done
