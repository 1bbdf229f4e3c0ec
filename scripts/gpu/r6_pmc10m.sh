#!/bin/bash
# Round 6: PMC passes of the 10M K=32 query kernel (BASELINE config 4)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6pmc10m
mkdir -p $O
bash tools/profile.sh pmc 32 10000000 > $O/pmc.txt 2>&1 || { echo PMC_FAIL; tail $O/pmc.txt; exit 1; }
cat $O/pmc.txt
