#!/bin/bash
# Distributed steady step replayed from a graph (opt-in) vs eager, world 1 RCCL, same box; the
# new graph test.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/graph
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -q -k "graph_replay or world1" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAIL; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for g in 0 1; do
    KN_DIST_GRAPH=$g timeout -k 10 180 python bench.py --dist > $O/d_${g}_$i.json 2> $O/d_${g}_$i.err || { echo FAIL; tail $O/d_${g}_$i.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/d_${g}_$i.json').read().strip().splitlines()[-1]);print('graph $g', round(d['ms_per_step'],4), d['check'], d['host_enqueue_ms_per_step'], d['invalid_async_steps'])"
  done
done
