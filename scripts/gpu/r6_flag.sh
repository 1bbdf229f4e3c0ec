#!/bin/bash
# Round 6: the deferred distributed step check fused into the exact kernel's last workgroup
# (KN_DIST_FUSED_FLAG, default on) -- distributed GPU tests + diag, then world-1 A/B vs the two
# separate flag kernels (KN_DIST_FUSED_FLAG=0)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6flag
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_distributed.py > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 300 python scripts/diag_dist_pipe.py > $O/diag.txt 2>&1 || { echo DIAG_FAIL; tail -30 $O/diag.txt; exit 1; }
tail -3 $O/diag.txt
: > $O/ab.txt
one() {  # label fused args...
  local label=$1 f=$2; shift 2
  KN_DIST_FUSED_FLAG=$f timeout -k 10 150 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('ms_query'), d.get('ms_route'))" >> $O/ab.txt
}
for pass in 1 2 3; do
  for f in 1 0; do
    one "fused=$f dist 200/50" $f --dist --steps 200 --warmup 50
    one "fused=$f dist 20/5" $f --dist --steps 20 --warmup 5
  done
done
one "engine 200/50" 1 --steps 200 --warmup 50
cat $O/ab.txt
