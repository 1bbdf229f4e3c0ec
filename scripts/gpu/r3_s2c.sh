#!/bin/bash
# Round 3 (session 2): x sub-cells on small clouds, ring order at K <= 16 (fixed A/B driver),
# host-API phase timings, PMC of the shipping query kernel.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2c
mkdir -p $O
timeout -k 10 300 python scripts/ab_xsub.py 20000 8,16 uniform,xyz:data/pts20K.xyz 20 1 2 > $O/ab_xsub_small.jsonl 2>> $O/err.log || { echo ABX_FAIL; tail -20 $O/err.log; exit 1; }
timeout -k 10 300 python scripts/ab_xsub.py 100000 8,16 uniform 12 1 2 >> $O/ab_xsub_small.jsonl 2>> $O/err.log || { echo ABX2_FAIL; tail -20 $O/err.log; exit 1; }
timeout -k 10 300 python scripts/ab_xsub.py 300000 16 uniform 12 1 2 >> $O/ab_xsub_small.jsonl 2>> $O/err.log || { echo ABX3_FAIL; tail -20 $O/err.log; exit 1; }
cat $O/ab_xsub_small.jsonl
timeout -k 10 300 python scripts/ab_multi.py ring 900000 8,16 uniform 12 > $O/ab_ring.jsonl 2>> $O/err.log || { echo ABR_FAIL; tail -20 $O/err.log; exit 1; }
cat $O/ab_ring.jsonl
KN_PREP_TIMING=1 timeout -k 10 100 ./bin/knn_cli --uniform 900000 --k 16 --api-bench 3 > $O/api.json 2> $O/api_phases.log || { echo API_FAIL; tail $O/api_phases.log; exit 1; }
cat $O/api.json; grep -v "^  \[\|HIP dev" $O/api_phases.log | tail -14
timeout -k 10 600 bash scripts/gpu/r3_pmc.sh > $O/pmc.log 2>&1 || { echo PMC_FAIL; tail -20 $O/pmc.log; exit 1; }
grep -v "^PMC" $O/pmc.log | head -60
