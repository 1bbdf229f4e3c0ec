#!/bin/bash
# Round 3 validation: GPU tests (single-GPU, C API incl. the C++ multi runtime, distributed) +
# pts20K / 900K benches + a kernel profile of each.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/val
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_a.log 2>&1 || { echo A_FAIL; tail -40 $O/pytest_a.log; exit 1; }
tail -1 $O/pytest_a.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_b.log 2>&1 || { echo B_FAIL; tail -40 $O/pytest_b.log; exit 1; }
tail -1 $O/pytest_b.log
timeout -k 10 200 python -u bench.py --xyz data/pts20K.xyz --k 8 --steps 200 --warmup 20 > $O/pts20k.json 2>$O/pts20k.err && cat $O/pts20k.json || exit 1
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 > $O/k16.json 2>$O/k16.err && cat $O/k16.json || exit 1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python3 $R/bench.py --steps 40 --warmup 5 > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail $R/$O/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof20 -o run -- python3 $R/bench.py --xyz $R/data/pts20K.xyz --k 8 --steps 100 --warmup 5 > $R/$O/prof20.log 2>&1 || { echo PROF_FAIL; tail $R/$O/prof20.log; exit 1; }
cd $R
python scripts/kernel_stats.py $(find $O/prof -name '*.db' | head -1) > $O/kstats.txt 2>&1; head -10 $O/kstats.txt
python scripts/kernel_stats.py $(find $O/prof20 -name '*.db' | head -1) > $O/kstats20.txt 2>&1; head -8 $O/kstats20.txt
