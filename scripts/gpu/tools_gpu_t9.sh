#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
: > gpurun_out/loopscale.jsonl
timeout -k 10 200 python bench.py --dist --steps 30 --warmup 5 > gpurun_out/_l.json 2>/dev/null || { echo DIST_FAIL; exit 1; }
tail -1 gpurun_out/_l.json >> gpurun_out/loopscale.jsonl
for w in 2 4 8; do
  timeout -k 10 300 python bench.py --loopback $w --n 900000 --k 16 --steps 10 --warmup 3 > gpurun_out/_l.json 2> gpurun_out/loop.err || { echo LOOP_FAIL $w; tail -5 gpurun_out/loop.err; exit 1; }
  tail -1 gpurun_out/_l.json >> gpurun_out/loopscale.jsonl
done
python -c "
import json
for l in open('gpurun_out/loopscale.jsonl'):
    d=json.loads(l); W=int(d['config'].get('parallelism','loopback1').replace('loopback','').replace('single','1') or 1)
    print(d['config']['parallelism'], round(d['ms_per_step'],3), 'per-rank ms', round(d['ms_per_step']/W,3), d.get('stats'), d.get('check'))"
