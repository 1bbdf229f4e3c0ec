#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5qsdbg
mkdir -p $O
KN_PIPE_QSTREAMS=2 KN_PIPE_UNROLL=2 AMD_LOG_LEVEL=3 timeout -k 10 120 python -X faulthandler bench.py --steps 4 --warmup 2 --no-check --n 100000 > $O/q2.json 2> $O/q2.err
echo "exit $?"
grep -v "^:3:" $O/q2.err | tail -40
grep "^:3:" $O/q2.err | tail -30
