#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5qsdbg
mkdir -p $O
KN_PIPE_QSTREAMS=2 timeout -k 10 120 python -X faulthandler bench.py --steps 200 --warmup 50 --no-check > $O/q2.json 2> $O/q2.err
echo "exit $?"
tail -60 $O/q2.err
