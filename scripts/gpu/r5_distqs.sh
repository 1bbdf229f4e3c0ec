#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5distqs2
mkdir -p $O
MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 RANK=0 WORLD_SIZE=1 timeout -k 10 400 python -u scripts/diag_dist_pipe.py 30 200000 > $O/diag.log 2>&1 || { echo DIAG_FAIL; tail -30 $O/diag.log; exit 1; }
grep -E "capture|ALL" $O/diag.log | cut -c1-200
p=29600
for rep in 1 2; do
for cfg in "1 0" "2 0" "2 1"; do
  set -- $cfg
  p=$((p+1))
  KN_DIST_QSTREAMS=$1 KN_DIST_CAPTURE=$2 MASTER_PORT=$p timeout -k 10 200 python bench.py --dist --steps 200 --warmup 50 --no-check > $O/d_q$1_c$2.json 2> $O/d_q$1_c$2.err || { echo DIST_FAIL; tail $O/d_q$1_c$2.err; exit 1; }
  echo "qs $1 capture $2: $(python -c "import json;d=json.loads(open('$O/d_q$1_c$2.json').read().splitlines()[-1]);print(round(d['ms_per_step'],4), d.get('dist_mode'))")"
done
done
KN_DIST_CAPTURE=0 MASTER_PORT=29690 timeout -k 10 200 python bench.py --dist --steps 20 --warmup 5 > $O/d20.json 2> $O/d20.err && echo "dist 20/5 eager qs2: $(python -c "import json;d=json.loads(open('$O/d20.json').read().splitlines()[-1]);print(round(d['ms_per_step'],4), d['check'])")"
timeout -k 10 200 python bench.py --steps 200 --warmup 50 --no-check > $O/eng.json 2> $O/eng.err && echo "engine $(python -c "import json;d=json.loads(open('$O/eng.json').read().splitlines()[-1]);print(round(d['ms_per_step'],4))")"
