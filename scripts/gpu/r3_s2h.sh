#!/bin/bash
# Round 3 (session 2): small-cloud step (pts20K, K=8; 100K K=16): one-workgroup build on/off,
# x sub-cells 1/2, pipelined vs serial steps.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2h
mkdir -p $O
: > $O/small.jsonl
for cfg in "data/pts20K.xyz 8" "data/pts20K.xyz 16"; do
  set -- $cfg
  for sb in 1 0; do for xs in 2 1; do for pl in "" "--no-pipeline"; do
    KN_SMALL_BUILD=$sb KN_XSUB=$xs timeout -k 10 120 python bench.py --xyz $1 --k $2 --steps 200 --warmup 20 $pl > $O/_l.json 2>> $O/err.log || { echo FAIL $cfg $sb $xs $pl; tail $O/err.log; exit 1; }
    python - "$1" "$2" "$sb" "$xs" "$pl" >> $O/small.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/s2h/_l.json") if l.startswith("{")][-1])
print(json.dumps({"cloud": sys.argv[1], "k": int(sys.argv[2]), "small_build": int(sys.argv[3]), "xsub": int(sys.argv[4]),
                  "pipelined": d.get("pipelined"), "ms_per_step": round(d["ms_per_step"], 4), "ms_build": d.get("ms_build"),
                  "ms_solve": d.get("ms_solve"), "check": d["check"]}))
PY
    tail -1 $O/small.jsonl
  done; done; done
done
timeout -k 10 300 python -u scripts/diag_checked_r3.py > $O/checked.log 2>&1 || { echo CHECKED_FAIL; tail -20 $O/checked.log; exit 1; }
tail -2 $O/checked.log
timeout -k 10 900 bash scripts/bench_suite.sh > $O/suite.log 2>&1 || { echo SUITE_FAIL; tail -20 $O/suite.log; exit 1; }
cp gpurun_out/bench_suite.jsonl $O/
cat $O/bench_suite.jsonl | cut -c1-250
