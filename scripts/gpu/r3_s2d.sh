#!/bin/bash
# Round 3 (session 2): engine with pooled streams / device blocks: GPU tests, smoke, bench,
# host-to-host API timing (staging + caches on / off) with prepare phase timers.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
cat $O/bench.json
for st in 0 1; do
  for k in 16 50; do
    KN_PREP_TIMING=1 KN_HOST_STAGE=$st KN_ARENA_CACHE=$st timeout -k 10 200 ./bin/knn_cli --uniform 900000 --k $k --api-bench 7 > $O/api${k}_s$st.json 2> $O/api${k}_s$st.log || { echo API_FAIL; tail $O/api${k}_s$st.log; exit 1; }
    echo "stage=$st $(cat $O/api${k}_s$st.json)"
  done
done
grep -h "allocate:\|release" $O/api16_s1.log | tail -6
