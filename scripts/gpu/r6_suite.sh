#!/bin/bash
# Round 6 checkpoint: GPU tests, smoke, then the BASELINE suite (scripts/bench_suite.sh)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6suite
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "PYTEST_FAIL"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1500 bash scripts/bench_suite.sh > $O/suite.log 2>&1 || { echo SUITE_FAIL; tail -30 $O/suite.log; exit 1; }
cp gpurun_out/bench_suite.jsonl $O/
python - <<'PY'
import json
for l in open("gpurun_out/r6suite/bench_suite.jsonl"):
    d = json.loads(l)
    print(f"{d['suite_label'][:60]:60s} {d['ms_per_step']:8.4f} ms  {d['value']:.3e} q/s  build {d.get('ms_build')} solve {d.get('ms_solve')} chk {d.get('check',{}).get('bad_rows', d.get('check',{}).get('bad_rows_all_ranks'))}")
PY
timeout -k 10 300 python scripts/diag_checked.py > $O/checked.log 2>&1 || { echo CHECKED_FAIL; tail -20 $O/checked.log; exit 1; }
tail -3 $O/checked.log
