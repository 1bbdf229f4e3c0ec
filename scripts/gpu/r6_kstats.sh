#!/bin/bash
# Round 6 end: kernel stats of the headline (900K K=16) and the reference K (K=50) bench steps
set -o pipefail
O=$PWD/gpurun_out/r6kstats
mkdir -p $O
bash tools/profile.sh kstats --steps 50 --warmup 20 > $O/k16.txt 2>&1 || { echo FAIL16; tail $O/k16.txt; exit 1; }
bash tools/profile.sh kstats --k 50 --steps 50 --warmup 20 > $O/k50.txt 2>&1 || { echo FAIL50; tail $O/k50.txt; exit 1; }
head -12 $O/k16.txt; head -12 $O/k50.txt
