#!/bin/bash
# kWin = 2 default: GPU suite + benches across K.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/winval1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for a in "--k 16" "--k 8" "--k 32" "--k 50" "--k 64" "--k 16" "--gen clustered"; do
  f=$O/b_$(echo $a | tr -d ' -').json
  timeout -k 10 180 python bench.py $a > $f 2> $f.err || { echo BENCH_FAIL $a; tail $f.err; exit 1; }
  python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$a', round(d['ms_per_step'],4), '%.3e' % d['value'], d['exact_path_queries'], d['check'])"
done
