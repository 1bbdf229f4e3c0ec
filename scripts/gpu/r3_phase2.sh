#!/bin/bash
# Round 3: per-phase cycle census of the query kernel (one-VGPR accumulator version) + baseline times.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/phase
mkdir -p $O
timeout -k 10 200 python scripts/phase_census.py 900000 8 16 32 50 64 > $O/census2.jsonl 2> $O/census2.err || { echo CENSUS_FAIL; tail $O/census2.err; exit 1; }
cat $O/census2.jsonl
timeout -k 10 200 python scripts/ab_variant.py phases 900000 16 10 > $O/ab16.txt 2>&1 || { echo AB_FAIL; tail $O/ab16.txt; exit 1; }
cat $O/ab16.txt
