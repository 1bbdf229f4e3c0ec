#!/bin/bash
# Round 3 (session 2): pipelined tree steps, small build opt-in: GPU suite, smoke, benches.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
: > $O/benches.jsonl
for a in "" "--gen clustered" "--gen surface" "--gen clustered --no-pipeline" "--gen surface --no-pipeline" "--xyz data/pts20K.xyz --k 8" "--xyz data/pts20K.xyz --k 8 --no-pipeline"; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 $a > $O/_b.json 2>> $O/err.log || { echo BENCH_FAIL $a; tail $O/err.log; exit 1; }
  python - "$a" >> $O/benches.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/s2i/_b.json") if l.startswith("{")][-1])
print(json.dumps({"args": sys.argv[1], "ms_per_step": round(d["ms_per_step"], 4), "value": d["value"], "ms_build": d.get("ms_build"),
                  "algo": d.get("query_algo"), "pipelined": d.get("pipelined"), "check": d["check"]}))
PY
  tail -1 $O/benches.jsonl
done
