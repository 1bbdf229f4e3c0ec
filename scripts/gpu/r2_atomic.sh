#!/bin/bash
# One-pass atomic steady router: distributed GPU tests + native/dist alternating on one box.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/atomic
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
run() { local name=$1; shift; timeout -k 10 240 python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);print('$name', round(d['ms_per_step'],4), d['check'], d.get('invalid_async_steps'))"; }
for i in 1 2 3; do run native_$i --no-check; run dist_$i --dist; run distdet_$i --dist --deterministic --no-check; done
run loop8 --loopback 8 --steps 10 --warmup 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_dist -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --no-check --steps 20 > $GRAFT_REPO_ROOT/$O/prof_dist.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo done
