#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
for k in 16 32 50; do
  timeout -k 10 300 python scripts/sweep_tiles.py 900000 $k 2.2,2.5,2.9,3.3,3.8,4.5 4x4x4 > gpurun_out/sweep3_k$k.log 2>&1 || { echo SWEEP_FAIL; tail gpurun_out/sweep3_k$k.log; exit 1; }
  echo "k=$k"; grep -v BEST gpurun_out/sweep3_k$k.log | grep '^{' | python -c "
import sys, json
for l in sys.stdin:
    r=json.loads(l); print(r['ppc'], r['halo'], r['cap'], r['ms'], r['exact'])"
done
