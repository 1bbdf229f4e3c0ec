#!/bin/bash
# Round 3: collect lane walk v2 (no-SLP build) vs round-2 lane walk built without (old) / with
# (oldslp) SLP vectorization. Smoke first, under short limits.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/collect2
mkdir -p $O
timeout -k 10 90 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python scripts/ab_multi.py old 900000 8,16,32,50 uniform 10 > $O/ab_old.jsonl 2> $O/ab.err || { echo AB_FAIL; tail -20 $O/ab.err; cat $O/ab_old.jsonl; exit 1; }
cat $O/ab_old.jsonl
timeout -k 10 300 python scripts/ab_multi.py oldslp 900000 16,50 uniform 10 > $O/ab_oldslp.jsonl 2>> $O/ab.err || { echo AB_FAIL; tail -20 $O/ab.err; exit 1; }
cat $O/ab_oldslp.jsonl
