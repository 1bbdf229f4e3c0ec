#!/bin/bash
# Binning plan A/B: points per streaming block (KN_BIN_ITEMS) x block size, 900K and 10M.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/binitems
mkdir -p $O
for n in 900000 10000000; do
for cfg in "4096 1024" "2048 1024" "8192 1024" "2048 512" "4096 1024" "2048 1024"; do
  set -- $cfg
  KN_BIN_ITEMS=$1 KN_BIN_THREADS=$2 timeout -k 10 200 python bench.py --no-check --n $n --steps 10 --warmup 2 > $O/b_${n}_$1_$2.json 2> $O/b_${n}_$1_$2.err || { echo FAIL; tail $O/b_${n}_$1_$2.err; exit 1; }
  echo "n $n items $1 threads $2 $(python -c "import json;d=json.load(open('$O/b_${n}_$1_$2.json'));print(round(d['ms_per_step'],4), d['ms_build'], d['ms_solve'])")"
done
done
