#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py "$@" 2>>gpurun_out/loop.err | grep '^{' >> gpurun_out/loop_r2.jsonl || { echo FAIL "$@"; tail -5 gpurun_out/loop.err; exit 1; }; }
run --loopback 8 --n 900000 --steps 10 --warmup 2
run --loopback 8 --n 900000 --steps 5 --warmup 1 --gen clustered
run --dist --n 900000 --steps 20 --warmup 3
cat gpurun_out/loop_r2.jsonl | cut -c1-900
