#!/bin/bash
# Round 3: adaptive halo boost -- distributed GPU tests + loopback 8x900K uniform / clustered.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/loop2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/loop.jsonl
for cfg in "uniform 2.5" "uniform 1.3" "clustered 2.5"; do
set -- $cfg
timeout -k 10 300 python -u bench.py --loopback 8 --n 900000 --k 16 --gen $1 --halo-factor $2 --steps 10 --warmup 6 > $O/l.json 2>>$O/loop.err || { echo FAIL $cfg; tail -20 $O/loop.err; exit 1; }
python - $1 $2 >> $O/loop.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/loop2/l.json") if l.startswith("{")][-1])
d["gen"], d["halo_factor"] = sys.argv[1], float(sys.argv[2])
print(json.dumps(d))
PY
python -c "
import json; d=json.loads(open('$O/loop.jsonl').readlines()[-1]); print(d['gen'], d['halo_factor'], round(d['ms_per_step'],3), d['stats'])"
done
