#!/bin/bash
# Round 3: phase census of the collect lane walk (_C_phases) vs the round-2 lane walk (_C_phasesold).
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/census
mkdir -p $O
timeout -k 10 120 python scripts/phase_census.py phases 900000 16 50 > $O/new.jsonl 2> $O/err.log || { echo FAIL; tail $O/err.log; exit 1; }
cat $O/new.jsonl
timeout -k 10 120 python scripts/phase_census.py phasesold 900000 16 50 > $O/old.jsonl 2>> $O/err.log || { echo FAIL; tail $O/err.log; exit 1; }
cat $O/old.jsonl
