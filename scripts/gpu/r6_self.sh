#!/bin/bash
# Round 6: the lane walk without a self slot (KN_SELF_SLOT=0, _C) vs with it (_C_self1); walk stats;
# the checked engine on the new code; the tile-kernel GPU tests
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6self
mkdir -p $O
timeout -k 10 120 python scripts/walk_stats.py 900000 16 32 50 8 > $O/ws.txt 2>&1 || { echo WS_FAIL; tail $O/ws.txt; }
grep -v amdgpu $O/ws.txt
for c in "uniform 16" "uniform 50" "uniform 8"; do
  KN_CHECKED=1 timeout -k 10 120 python scripts/diag_engine_k.py $c > $O/chk_$(echo $c | tr ' ' _).txt 2>&1 || { echo "DIAG_FAIL checked $c"; tail -5 $O/chk_$(echo $c | tr ' ' _).txt; exit 1; }
  grep -v amdgpu.ids $O/chk_$(echo $c | tr ' ' _).txt | grep -E "debug_words after pipe|rows equal" | cut -c1-200
done
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_reference_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { echo "PYTEST_FAIL"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
: > $O/ab.txt
for k in 16 50 32 8 64; do
  echo "== self1 k=$k" >> $O/ab.txt
  timeout -k 10 200 python scripts/ab_variant.py self1 900000 $k 12 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $k"; tail $O/ab.txt; exit 1; }
done
cat $O/ab.txt
