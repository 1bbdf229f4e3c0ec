#!/bin/bash
# PMC passes on the query kernel (each pass its own run; <= 8 SQ counters per pass)
set -o pipefail
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$PWD
export PYTHONPATH=$R
timeout -k 10 120 python scripts/diag_work.py 900000 16 > gpurun_out/diag_work.json 2>&1 || { echo DIAG_FAIL; tail gpurun_out/diag_work.json; exit 1; }
cat gpurun_out/diag_work.json
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc/counters_list.txt 2>&1 || echo LIST_FAIL
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d $R/gpurun_out/pmc/p$i -o run -- python3 $R/scripts/prof_query.py 900000 16 2 > $R/gpurun_out/pmc/p$i.log 2>&1 || { echo PMC${i}_FAIL; tail -5 $R/gpurun_out/pmc/p$i.log; exit 1; }
  echo PMC${i}_OK
done
cd $R
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_native -o run -- python3 $R/bench.py --no-check --steps 30 --warmup 5 > $R/gpurun_out/prof_native.log 2>&1 || { echo PROF_FAIL; tail $R/gpurun_out/prof_native.log; exit 1; }
echo PROF_OK
