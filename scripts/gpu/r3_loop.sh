#!/bin/bash
# Round 3: loopback (8 virtual ranks on one GPU) vs halo factor, uniform and clustered, with
# device forwarding in the steady steps.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/loop
mkdir -p $O
: > $O/loop.jsonl
for gen in uniform clustered; do
for hf in 2.5 1.3 1.0; do
timeout -k 10 300 python -u bench.py --loopback 8 --n 900000 --k 16 --gen $gen --halo-factor $hf --steps 10 --warmup 3 > $O/l.json 2>>$O/loop.err || { echo FAIL $gen $hf; tail -20 $O/loop.err; exit 1; }
python - $gen $hf >> $O/loop.jsonl <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/loop/l.json") if l.startswith("{")][-1])
d["gen"], d["halo_factor"] = sys.argv[1], float(sys.argv[2])
print(json.dumps(d))
PY
tail -1 $O/loop.jsonl | cut -c1-400
done
done
