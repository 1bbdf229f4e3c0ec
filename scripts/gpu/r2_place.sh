#!/bin/bash
# Direct placement of the own segment in steady distributed steps: GPU suite, world-1 RCCL
# bench, loopback 8 x 900K, trace of the distributed step.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/place
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2 3; do
  timeout -k 10 180 python bench.py --dist > $O/dist_$i.json 2> $O/dist_$i.err || { echo DIST_FAIL; tail $O/dist_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/dist_$i.json').read().strip().splitlines()[-1]);print('dist', round(d['ms_per_step'],4), d['check'], d['invalid_async_steps'])"
done
timeout -k 10 300 python bench.py --loopback 8 --steps 10 --warmup 3 > $O/loop8.json 2> $O/loop8.err || { echo LOOP_FAIL; tail $O/loop8.err; exit 1; }
python -c "import json;d=json.loads(open('$O/loop8.json').read().strip().splitlines()[-1]);print('loop8', round(d['ms_per_step'],4), d['check'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_dist -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --no-check --steps 20 > $GRAFT_REPO_ROOT/$O/prof_dist.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo done
