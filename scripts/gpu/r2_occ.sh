#!/bin/bash
# Occupancy sensitivity of the query kernel: pad the workgroup LDS (39.5 KB -> 4 WGs/CU) to
# 3 WGs/CU (+14 KB) and 2 WGs/CU (+41 KB); K=16 and K=50 solve times.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/occ
mkdir -p $O
for k in 16 50; do
  for pad in 0 14000 41000 0 14000; do
    KN_LDS_EXTRA=$pad timeout -k 10 120 python bench.py --k $k --no-check > $O/k${k}_$pad.json 2> $O/k${k}_$pad.err || { echo FAIL; tail $O/k${k}_$pad.err; exit 1; }
    echo "k $k pad $pad $(python -c "import json;d=json.load(open('$O/k${k}_$pad.json'));print(round(d['ms_per_step'],4), d['ms_solve'])")"
  done
done
