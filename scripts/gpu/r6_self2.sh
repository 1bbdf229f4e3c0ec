#!/bin/bash
# Round 6: repeat of the self-slot A/B (K=50 / 64 / 16), 16 rounds each, with the GPU clock logged
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6self2
mkdir -p $O
(rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|mclk|Power|Temp" | head -8) > $O/smi_before.txt || true
: > $O/ab.txt
for k in 50 64 16 50; do
  echo "== self1 k=$k" >> $O/ab.txt
  timeout -k 10 200 python scripts/ab_variant.py self1 900000 $k 16 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $k"; tail $O/ab.txt; exit 1; }
done
(rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -E "sclk|mclk|Power|Temp" | head -8) > $O/smi_after.txt || true
cat $O/ab.txt; cat $O/smi_before.txt $O/smi_after.txt
