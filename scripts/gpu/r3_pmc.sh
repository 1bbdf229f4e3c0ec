#!/bin/bash
# Round 3 PMC of the shipping query kernel (K=16 and K=50, 900K uniform): every pass runs the same
# driver (1 build + 3 query dispatches), one counter group per run (<= 8 SQ, <= 4 TCC), so every
# counter averages over the same 3 dispatches (round-2 verdict: mixed dispatch counts).
set -o pipefail
R=$PWD
export PYTHONPATH=$R TMPDIR=/tmp
O=$R/gpurun_out/pmc3
mkdir -p $O
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_WAVES SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
P3="SQ_WAVES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32"
P4="FETCH_SIZE"
P5="TCC_HIT_sum TCC_MISS_sum"
for K in 16 50; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d $O/k${K}_p$i -o run -- python3 $R/scripts/prof_query.py 900000 $K 3 > $O/k${K}_p$i.log 2>&1 || { echo PMC_K${K}_P${i}_FAIL; tail -5 $O/k${K}_p$i.log; exit 1; }
    echo PMC_K${K}_P${i}_OK
  done
  python3 $R/scripts/pmc_summary.py knn_tile_kernel $(find $O -path "*k${K}_p*" -name "*.db") > $O/summary_k$K.txt 2>&1 || true
  cat $O/summary_k$K.txt
done
