#!/bin/bash
# A/B of the split top-K insertion networks (KN_TOPK_SPLIT 1 / 2 vs 0), query kernel only,
# interleaved in process (scripts/ab_variant.py), then the second-query-stream crash debug.
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5split
mkdir -p $O
for k in 16 32 50 64; do
  for v in split1 split2; do
    echo "k=$k $v: $(timeout -k 10 120 python scripts/ab_variant.py $v 900000 $k 15 2>&1 | tr '\n' ' ')"
  done
done | tee $O/ab.txt
bash scripts/gpu/r5_qs_dbg.sh
