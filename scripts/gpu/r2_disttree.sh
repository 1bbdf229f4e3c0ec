#!/bin/bash
# Tree path for refined (non-uniform) shares in the distributed local solve. The bounds-checked
# build runs first (violations are redirected and reported instead of faulting); the release
# suite only runs if it is clean.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/disttree
mkdir -p $O
timeout -k 10 400 python -u scripts/diag_checked.py > $O/checked.log 2>&1 || { echo CHECKED_FAIL; grep -v amdgpu.ids $O/checked.log | tail; exit 1; }
grep -v amdgpu.ids $O/checked.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
run() { local name=$1; shift; timeout -k 10 600 python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);print('$name', round(d['ms_per_step'],4), d['check'], d.get('stats'))"; }
run loop8_clustered --loopback 8 --gen clustered --steps 5 --warmup 2
run loop8_uniform --loopback 8 --steps 10 --warmup 3
echo done
