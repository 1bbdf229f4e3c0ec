#!/bin/bash
# Generic check after a kernel/runtime change: full GPU test suite, native + distributed(world 1)
# headline bench, and rocprofv3 kernel stats of the native bench.  usage: tools_gpu_check.sh LABEL
set -o pipefail
L=${1:-check}
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
R=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${L}_tests.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/${L}_tests.log; exit 1; }
tail -2 gpurun_out/${L}_tests.log
timeout -k 10 200 python bench.py --n 900000 --k 16 --steps 50 --warmup 10 > gpurun_out/${L}_native.json 2> gpurun_out/${L}_native.err || { echo NATIVE_FAIL; tail gpurun_out/${L}_native.err; exit 1; }
tail -1 gpurun_out/${L}_native.json | cut -c1-330
timeout -k 10 200 python bench.py --dist --n 900000 --k 16 --steps 50 --warmup 10 > gpurun_out/${L}_dist.json 2> gpurun_out/${L}_dist.err || { echo DIST_FAIL; tail gpurun_out/${L}_dist.err; exit 1; }
tail -1 gpurun_out/${L}_dist.json | cut -c1-330
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${L}_prof -o run -- python3 $R/bench.py --no-check --steps 30 --warmup 5 > $R/gpurun_out/${L}_prof.log 2>&1 || { echo PROF_FAIL; tail $R/gpurun_out/${L}_prof.log; exit 1; }
cd $R
python scripts/kernel_stats.py $(find gpurun_out/${L}_prof -name "*.db" | head -1) 16 > gpurun_out/${L}_kstats.txt && cat gpurun_out/${L}_kstats.txt
