#!/bin/bash
mkdir -p gpurun_out
KN_CHECKED=1 PYTHONPATH=. timeout -k 5 60 python scripts/diag_bench.py 100000 > gpurun_out/diag_bench.log 2>&1
rc=$?; echo "diag rc=$rc"; tail -30 gpurun_out/diag_bench.log
