#!/bin/bash
# PMC passes on the shipping query kernel (lane walk + window re-rank) at K=16 and K=50, one
# counter group per run (<= 8 SQ, <= 4 TCC), plus kernel stats of the default bench.
set -o pipefail
R=$PWD
export PYTHONPATH=$R TMPDIR=/tmp
mkdir -p gpurun_out/pmc2
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
P3="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32"
P4="FETCH_SIZE"
P5="TCC_HIT_sum TCC_MISS_sum"
for K in 16 50; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d $R/gpurun_out/pmc2/k${K}_p$i -o run -- python3 $R/scripts/prof_query.py 900000 $K 2 > $R/gpurun_out/pmc2/k${K}_p$i.log 2>&1 || { echo PMC_K${K}_P${i}_FAIL; tail -5 $R/gpurun_out/pmc2/k${K}_p$i.log; exit 1; }
    echo PMC_K${K}_P${i}_OK
  done
done
cd $R
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench_r2 -o run -- python3 $R/bench.py --no-check --steps 30 --warmup 5 > $R/gpurun_out/prof_bench_r2.log 2>&1 || { echo PROF_FAIL; tail $R/gpurun_out/prof_bench_r2.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench_r2_k50 -o run -- python3 $R/bench.py --no-check --k 50 --steps 20 --warmup 3 > $R/gpurun_out/prof_bench_r2_k50.log 2>&1 || { echo PROF50_FAIL; tail $R/gpurun_out/prof_bench_r2_k50.log; exit 1; }
echo PROF_OK
