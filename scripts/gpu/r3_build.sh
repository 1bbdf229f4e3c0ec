#!/bin/bash
# Round 3: one-workgroup small-cloud build + batched build loads: GPU tests, pts20K A/B, 900K profile.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/build
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo GPU_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in 1 0; do KN_SMALL_BUILD=$v timeout -k 10 200 python -u bench.py --xyz data/pts20K.xyz --k 8 --steps 200 --warmup 20 > $O/small_$v.json 2>$O/small_$v.err || exit 1; cat $O/small_$v.json; done
timeout -k 10 200 python -u bench.py --steps 50 --warmup 10 > $O/bench_k16.json 2>$O/bench_k16.err && cat $O/bench_k16.json || exit 1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python3 $R/bench.py --steps 40 --warmup 5 > $R/$O/prof.log 2>&1 || { echo PROF_FAIL; tail $R/$O/prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof20 -o run -- python3 $R/bench.py --xyz $R/data/pts20K.xyz --k 8 --steps 100 --warmup 5 > $R/$O/prof20.log 2>&1 || { echo PROF_FAIL; tail $R/$O/prof20.log; exit 1; }
cd $R
python scripts/kernel_stats.py $(find $O/prof -name '*.db' | head -1) > $O/kstats.txt 2>&1; head -12 $O/kstats.txt
python scripts/kernel_stats.py $(find $O/prof20 -name '*.db' | head -1) > $O/kstats20.txt 2>&1; head -8 $O/kstats20.txt
