#!/bin/bash
# GPU box: stream-vs-tile query kernel A/B (checked build first: OOB accesses are reported, not faulted)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
O=gpurun_out/ab.log
: > $O
timeout -k 10 120 python scripts/ab_algo.py 100000 16 2 _C_checked uniform >> $O 2>&1 || { echo CHK_FAIL; tail -5 $O; exit 1; }
timeout -k 10 120 python scripts/ab_algo.py 100000 50 2 _C_checked clustered >> $O 2>&1 || { echo CHK2_FAIL; tail -5 $O; exit 1; }
timeout -k 10 120 python scripts/ab_algo.py 900000 16 10 _C >> $O 2>&1 || { echo AB_FAIL; tail -5 $O; exit 1; }
timeout -k 10 120 python scripts/ab_algo.py 900000 16 10 _C_wpe6 >> $O 2>&1 || { echo AB6_FAIL; tail -5 $O; exit 1; }
timeout -k 10 120 python scripts/ab_algo.py 900000 16 10 _C_wpe4 >> $O 2>&1 || { echo AB4_FAIL; tail -5 $O; exit 1; }
timeout -k 10 120 python scripts/ab_algo.py 900000 32 10 _C >> $O 2>&1 || { echo AB32_FAIL; tail -5 $O; exit 1; }
timeout -k 10 120 python scripts/ab_algo.py 900000 8 10 _C >> $O 2>&1 || { echo AB8_FAIL; tail -5 $O; exit 1; }
grep -v amdgpu.ids $O
