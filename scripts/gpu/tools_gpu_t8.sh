#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 500 python scripts/sweep_tiles.py 900000 16 3.0,3.4,3.9 4x4x4,4x4x2,8x4x4,4x4x8,8x8x4,4x8x8,6x6x6,4x4x6,6x4x4,2x4x4,8x4x2,4x8x4 > gpurun_out/sweep4.log 2>&1 || { echo SWEEP_FAIL; tail gpurun_out/sweep4.log; exit 1; }
grep '^{' gpurun_out/sweep4.log | python -c "
import sys, json
rows=[json.loads(l) for l in sys.stdin]
rows.sort(key=lambda r: r['ms'])
for r in rows[:14]: print(r['ppc'], r['tile'], r['halo'], r['cap'], r['lds'], r['ms'], r['exact'], r['dense'])"
