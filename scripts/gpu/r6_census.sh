#!/bin/bash
# Round 6: where the K=16 / K=50 query kernel spends its waves now (phase census, KN_PHASES
# build) and the PMC of the shipped K=16 kernel after the re-rank changes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6census
mkdir -p $O
timeout -k 10 120 python scripts/phase_census.py phases 900000 16 50 > $O/census.txt 2>&1 || { echo CENSUS_FAIL; tail $O/census.txt; exit 1; }
grep -v amdgpu $O/census.txt
bash tools/profile.sh pmc 16 900000 > $O/pmc_k16.txt 2>&1 || { echo "PMC_FAIL"; tail $O/pmc_k16.txt; exit 1; }
grep -E "per wave|/ WAVE|conflict|vgpr" $O/pmc_k16.txt
