#!/bin/bash
# Round 2, first GPU call: GPU tests, headline bench (K=16) + K=50 bench, counter list, and PMC
# passes on the SHIPPING lane-walk kernel (knn_tile_kernel<KT,2,true>) at K=16 and K=50.
set -o pipefail
R=$PWD
export PYTHONPATH=$R
mkdir -p gpurun_out/pmc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python bench.py > gpurun_out/bench_k16.json 2> gpurun_out/bench_k16.err || { echo BENCH_FAIL; tail gpurun_out/bench_k16.err; exit 1; }
cat gpurun_out/bench_k16.json
timeout -k 10 120 python bench.py --k 50 > gpurun_out/bench_k50.json 2> gpurun_out/bench_k50.err || { echo BENCH50_FAIL; tail gpurun_out/bench_k50.err; exit 1; }
cat gpurun_out/bench_k50.json
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/pmc/counters_list.txt 2>&1 || echo LIST_FAIL
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
for K in 16 50; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d $R/gpurun_out/pmc/k${K}_p$i -o run -- python3 $R/scripts/prof_query.py 900000 $K 2 > $R/gpurun_out/pmc/k${K}_p$i.log 2>&1 || { echo PMC_K${K}_P${i}_FAIL; tail -5 $R/gpurun_out/pmc/k${K}_p$i.log; exit 1; }
    echo PMC_K${K}_P${i}_OK
  done
done
cd $R
ls -R gpurun_out/pmc | head -50
