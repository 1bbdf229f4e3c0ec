#!/bin/bash
# Round 6: PMC passes of the K=16 and K=50 query kernels (900K uniform)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6pmc
mkdir -p $O
bash tools/profile.sh pmc 16 900000 > $O/pmc16.txt 2>&1 || { echo PMC16_FAIL; tail $O/pmc16.txt; exit 1; }
bash tools/profile.sh pmc 50 900000 > $O/pmc50.txt 2>&1 || { echo PMC50_FAIL; tail $O/pmc50.txt; exit 1; }
cat $O/pmc16.txt
