#!/bin/bash
# round-end rehearsal: smoke(), default bench.py (driver contract), rocprofv3 kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
R=$PWD
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { echo BENCH_FAIL; tail gpurun_out/final_bench.err; exit 1; }
tail -1 gpurun_out/final_bench.json
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/final_prof -o run -- python3 $R/bench.py --no-check --steps 30 --warmup 5 > $R/gpurun_out/final_prof.log 2>&1 || { echo PROF_FAIL; tail $R/gpurun_out/final_prof.log; exit 1; }
cd $R
python scripts/kernel_stats.py $(find gpurun_out/final_prof -name "*.db" | head -1) 16 > gpurun_out/final_kstats.txt && cat gpurun_out/final_kstats.txt
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/final_prof50 -o run -- python3 $R/bench.py --no-check --k 50 --steps 20 --warmup 5 > $R/gpurun_out/final_prof50.log 2>&1 || { echo PROF50_FAIL; tail $R/gpurun_out/final_prof50.log; exit 1; }
cd $R
python scripts/kernel_stats.py $(find gpurun_out/final_prof50 -name "*.db" | head -1) 16 > gpurun_out/final_kstats_k50.txt && cat gpurun_out/final_kstats_k50.txt
