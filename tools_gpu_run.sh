#!/bin/bash
mkdir -p gpurun_out
run() { local name=$1; local t=$2; shift 2; PYTHONPATH=. timeout -k 5 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -${TAILN:-3} gpurun_out/$name.log; return $rc; }
run bench 180 python bench.py --steps 20 --warmup 5 || exit 1
TAILN=6 run pytest_gpu 600 python -m pytest tests/test_gpu.py -q -x -p no:cacheprovider --timeout 300 -m gpu || exit 1
