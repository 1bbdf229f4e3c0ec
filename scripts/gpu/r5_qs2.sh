#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5qs2
mkdir -p $O
for rep in 1 2; do
for cfg in "1 10" "2 2" "2 0" "1 0"; do
  set -- $cfg
  KN_PIPE_QSTREAMS=$1 KN_PIPE_UNROLL=$2 timeout -k 10 120 python bench.py --steps 200 --warmup 50 --no-check > $O/q$1_u$2.json 2> $O/q$1_u$2.err
  rc=$?
  echo "qs $1 unroll $2 rc $rc $(python -c "import json;d=json.loads(open('$O/q$1_u$2.json').read().splitlines()[-1]);print(round(d['ms_per_step'],4))" 2>/dev/null)"
  if [ $rc -ne 0 ]; then tail -5 $O/q$1_u$2.err; exit 1; fi
  KN_PIPE_QSTREAMS=$1 KN_PIPE_UNROLL=$2 timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $O/d$1_u$2.json 2> $O/d$1_u$2.err || exit 1
  echo "   20/5: $(python -c "import json;d=json.loads(open('$O/d$1_u$2.json').read().splitlines()[-1]);print(round(d['ms_per_step'],4), d['check'])" 2>/dev/null)"
done
done
KN_PIPE_QSTREAMS=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py -x -q --timeout 200 --timeout-method thread -k "stream or unrolled or pipeline" > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
