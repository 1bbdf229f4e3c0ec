#!/bin/bash
# Round 6 checkpoint: full GPU suite, then PMC passes of the K=16 and K=50 query kernels
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6check
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
bash tools/profile.sh pmc 16 900000 > $O/pmc16.txt 2>&1 || { echo PMC16_FAIL; tail $O/pmc16.txt; exit 1; }
bash tools/profile.sh pmc 50 900000 > $O/pmc50.txt 2>&1 || { echo PMC50_FAIL; tail $O/pmc50.txt; exit 1; }
head -40 $O/pmc16.txt
