#!/bin/bash
mkdir -p gpurun_out
run() { local name=$1; local t=$2; shift 2; PYTHONPATH=. timeout -k 5 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -14 gpurun_out/$name.log; return $rc; }
run bench 180 python bench.py --steps 20 --warmup 5 || exit 1
run bench_k50 180 python bench.py --steps 10 --warmup 3 --k 50 --no-check || exit 1
run pytest_gpu 600 python -m pytest tests/test_gpu.py tests/test_capi.py -q -p no:cacheprovider --timeout 300 -m gpu || exit 1
