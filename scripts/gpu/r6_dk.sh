#!/bin/bash
# Round 6: K-th distance taken from the buffered row position (KN_VEC_DK) vs the per-entry
# position compare (_C_nodk): GPU grid tests, query A/B (rows identical)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6dk
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
: > $O/ab.txt
for k in 16 50 32 16 50; do
  echo "== nodk k=$k" >> $O/ab.txt
  timeout -k 10 200 python scripts/ab_variant.py nodk 900000 $k 14 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $k"; exit 1; }
done
cat $O/ab.txt
