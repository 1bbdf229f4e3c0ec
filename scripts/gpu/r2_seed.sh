#!/bin/bash
# Exact kernel seeded with the tile kernel's K-th distance: GPU suite + K=50/64/clustered-grid
# benches + kernel stats at K=64.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/seed
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for a in "--k 50" "--k 64" "--k 50" "--k 64" "--k 16" "--gen clustered --algo grid"; do
  f=$O/b_$(echo $a | tr -d ' -').json
  timeout -k 10 180 python bench.py $a > $f 2> $f.err || { echo BENCH_FAIL $a; tail $f.err; exit 1; }
  python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$a', round(d['ms_per_step'],4), d['ms_solve'], d['exact_path_queries'], d['check'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_k64 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --k 64 --steps 20 > $GRAFT_REPO_ROOT/$O/prof_k64.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo done
