#!/bin/bash
# Round 3 (session 2): grouped tree traversal (G = 4 / 2 groups per wave) vs the wave-wide one.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2j
mkdir -p $O
for v in tg4 tg2; do
  timeout -k 10 400 python scripts/ab_tree.py $v 900000 16,50 clustered,surface,uniform 6 > $O/ab_$v.jsonl 2>> $O/err.log || { echo AB_FAIL $v; tail -20 $O/err.log; cat $O/ab_$v.jsonl; exit 1; }
  cat $O/ab_$v.jsonl
done
: > $O/prio.txt
for r in 1 2; do for pr in 0 1; do
  KN_PIPE_PRIO=$pr timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-check > $O/_p.json 2>> $O/err.log || { echo PRIO_FAIL; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/_p.json') if l.startswith('{')][-1]); print('prio=$pr', round(d['ms_per_step'],4), '%.3e' % d['value'])" >> $O/prio.txt
done; done
cat $O/prio.txt
