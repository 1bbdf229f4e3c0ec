#!/bin/bash
# Round 4: PMC passes on knn_tree_kernel (900K clustered, K=16): issue vs wait breakdown
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4pmc_tree
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD"
P3="TCC_HIT_sum TCC_MISS_sum"
i=0
dbs=()
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d "$O/p$i" -o run -- python3 "$R/scripts/prof_tree.py" 900000 16 clustered 2 > "$O/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$O/p$i.log"; exit 1; }
  dbs+=("$(find "$O/p$i" -name "*.db" | head -1)")
done
python3 "$R/scripts/pmc_summary.py" knn_tree_kernel "${dbs[@]}" > "$O/summary.txt"
cat "$O/summary.txt"
