#!/bin/bash
# Round 3 (session 2): kernel stats of the tree path (clustered / surface clouds, pipelined steps).
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2o
mkdir -p $O
for g in clustered surface; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/p_$g -o run -- python3 $GRAFT_REPO_ROOT/bench.py --gen $g --steps 20 --warmup 5 --no-check > $GRAFT_REPO_ROOT/$O/p_$g.log 2>&1) || { echo PROF_FAIL $g; tail $O/p_$g.log; exit 1; }
  python scripts/kernel_stats.py $(find $O/p_$g -name '*.db' | head -1) 16 > $O/kstats_$g.txt 2>&1; head -8 $O/kstats_$g.txt
done

# bench step-count sensitivity of the default (pipelined) headline: short runs vs steady state
: > $O/steps.txt
for sw in "20 5" "100 20" "200 20" "20 5" "200 20"; do
  set -- $sw
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-check > $O/_b.json 2>> $O/err.log || { echo BENCH_FAIL; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/_b.json') if l.startswith('{')][-1]); print('steps $1 warmup $2', round(d['ms_per_step'],4), '%.3e' % d['value'])" >> $O/steps.txt
done
cat $O/steps.txt
echo done
