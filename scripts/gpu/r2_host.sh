#!/bin/bash
# Is the distributed steady step host-bound? host enqueue time vs step time (world 1, RCCL),
# plus the 2-rank gloo host-staged rehearsal on one GPU.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/host
mkdir -p $O
for i in 1 2; do
  timeout -k 10 180 python bench.py --dist --no-check > $O/dist_$i.json 2> $O/dist_$i.err || { echo FAIL; tail $O/dist_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/dist_$i.json').read().strip().splitlines()[-1]);print('dist', round(d['ms_per_step'],4), 'host enqueue', d['host_enqueue_ms_per_step'])"
done
