#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/abbuild
mkdir -p $O
: > $O/ab2.jsonl
for v in batch0 regs0 bbox256; do
timeout -k 10 300 python -u scripts/ab_build.py $v 300000,900000,12500000 16 10 >> $O/ab2.jsonl 2>$O/ab.err || { tail $O/ab.err; exit 1; }
done
cat $O/ab2.jsonl
timeout -k 10 300 python -u scripts/ab_multi.py win0 900000 8,16 xyz:data/pts20K.xyz 10 > $O/ab_pts20k.jsonl 2>$O/ab.err || { tail $O/ab.err; exit 1; }
timeout -k 10 300 python -u scripts/ab_multi.py win0 900000 8,16,32,50 uniform 10 >> $O/ab_pts20k.jsonl 2>>$O/ab.err || { tail $O/ab.err; exit 1; }
timeout -k 10 300 python -u scripts/ab_multi.py win0 100000 8,16 uniform 10 >> $O/ab_pts20k.jsonl 2>>$O/ab.err || { tail $O/ab.err; exit 1; }
cat $O/ab_pts20k.jsonl
