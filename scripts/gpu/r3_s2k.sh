#!/bin/bash
# Round 3 (session 2): after the rank_local refactor: the GPU suite; pipelined-step build-stream
# priority A/B; the distributed path at world 1 vs native.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
: > $O/prio.txt
for r in 1 2; do for pr in 0 1; do
  KN_PIPE_PRIO=$pr timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-check > $O/_p.json 2>> $O/err.log || { echo PRIO_FAIL; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/_p.json') if l.startswith('{')][-1]); print('prio=$pr', round(d['ms_per_step'],4), '%.3e' % d['value'])" >> $O/prio.txt
done; done
cat $O/prio.txt
timeout -k 10 200 python bench.py --dist --steps 30 --warmup 5 > $O/bench_dist1.json 2> $O/bench_dist1.err || { echo DIST_FAIL; tail $O/bench_dist1.err; exit 1; }
tail -c 700 $O/bench_dist1.json
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-pipeline > $O/bench_serial.json 2>> $O/err.log || { echo SER_FAIL; exit 1; }
tail -c 300 $O/bench_serial.json
