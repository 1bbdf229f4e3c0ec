#!/bin/bash
# Round 3: second re-rank window (KN_WIN2) A/B + one-workgroup small build.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/small
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo GPU_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -m pytest tests/test_capi.py tests/test_gpu_distributed.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_capi.log 2>&1 || { echo CAPI_FAIL; tail -30 $O/pytest_capi.log; exit 1; }
tail -1 $O/pytest_capi.log
timeout -k 10 300 python -u scripts/ab_multi.py win0 900000 8,16 xyz:data/pts20K.xyz 10 > $O/ab_pts20k.jsonl 2>$O/ab.err || { tail $O/ab.err; exit 1; }
cat $O/ab_pts20k.jsonl
timeout -k 10 300 python -u scripts/ab_multi.py win0 900000 8,16,32,50 uniform,clustered 10 >> $O/ab_900k.jsonl 2>>$O/ab.err || { tail $O/ab.err; exit 1; }
cat $O/ab_900k.jsonl
for v in 1 0; do KN_SMALL_BUILD=$v timeout -k 10 200 python -u bench.py --xyz data/pts20K.xyz --k 8 --steps 200 --warmup 20 > $O/small_$v.json 2>$O/small_$v.err || exit 1; cat $O/small_$v.json; done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof20 -o run -- python3 $R/bench.py --xyz $R/data/pts20K.xyz --k 8 --steps 100 --warmup 5 > $R/$O/prof20.log 2>&1 || { echo PROF_FAIL; tail $R/$O/prof20.log; exit 1; }
cd $R
python scripts/kernel_stats.py $(find $O/prof20 -name '*.db' | head -1) > $O/kstats20.txt 2>&1; head -8 $O/kstats20.txt
