#!/bin/bash
# Round 5: the distributed pipeline in graph / eager / injected-capture-failure modes at world 1
# (scripts/diag_dist_pipe.py), the engine's stream-after-unrolled race test, headline bench, and the
# world-1 distributed bench in graph and eager modes.
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${OUT_DIR:-r5dist}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py -x -v --timeout 120 --timeout-method thread -k "stream" > $O/pytest_stream.log 2>&1 || { echo STREAM_FAIL; tail -30 $O/pytest_stream.log; exit 1; }
tail -2 $O/pytest_stream.log
MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 WORLD_SIZE=1 timeout -k 10 400 python -u scripts/diag_dist_pipe.py 30 200000 > $O/diag_dist_pipe.log 2>&1 || { echo DIAG_FAIL; tail -30 $O/diag_dist_pipe.log; exit 1; }
cat $O/diag_dist_pipe.log
timeout -k 10 200 python bench.py --steps 200 --warmup 50 --no-check > $O/bench_200.json 2> $O/bench_200.err || { echo BENCH_FAIL; tail $O/bench_200.err; exit 1; }
cat $O/bench_200.json
for cap in 1 0 1 0; do
  KN_DIST_CAPTURE=$cap MASTER_PORT=$((29570 + cap)) timeout -k 10 200 python bench.py --dist --steps 200 --warmup 50 --no-check > $O/dist_cap$cap.json 2> $O/dist_cap$cap.err || { echo DIST_FAIL; tail $O/dist_cap$cap.err; exit 1; }
  cat $O/dist_cap$cap.json
done
KN_DIST_CAPTURE=0 MASTER_PORT=29575 timeout -k 10 200 python bench.py --dist --steps 20 --warmup 5 > $O/dist_eager_20.json 2> $O/dist_eager_20.err || { echo DIST_FAIL; tail $O/dist_eager_20.err; exit 1; }
cat $O/dist_eager_20.json
echo done
