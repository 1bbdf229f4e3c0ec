#!/bin/bash
# Round 4: isolate a failing local flag of the loopback DistPipeline (fused router x halo field)
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4diag
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
for fused in 1; do
  for fg in 64 0; do
    echo "== fused $fused field $fg"
    KN_ROUTE_FUSED=$fused timeout -k 10 120 python3 scripts/diag_loopback_pipe.py 2 uniform $fg 2>&1 | grep -v "NCCL WARN" | tail -4 || exit 1
  done
done
