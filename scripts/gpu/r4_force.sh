#!/bin/bash
# Round 4: where the forced-collective world-1 native pipeline crashes.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4force
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
KN_DIAG_VERBOSE=1 NCCL_DEBUG=WARN MASTER_PORT=$((29700 + RANDOM % 100)) timeout -k 10 120 python3 -X faulthandler scripts/diag_dist_pipe.py 5 200000 1 > "$O/force.log" 2>&1
echo "rc $?"
tail -40 "$O/force.log"
