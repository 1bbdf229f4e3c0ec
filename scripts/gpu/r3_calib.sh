#!/bin/bash
# Round 3: VALU issue-rate calibration (csrc/tools/valu_rate.hip) + default bench.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/calib
mkdir -p $O
timeout -k 10 120 ./bin/valu_rate 20000 > $O/valu_rate.jsonl 2> $O/valu_rate.err || { echo VALU_FAIL; cat $O/valu_rate.err; exit 1; }
cat $O/valu_rate.jsonl
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail $O/bench.err; exit 1; }
cat $O/bench.json
