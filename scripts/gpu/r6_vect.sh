#!/bin/bash
# Round 6: tree-path row stores, V positions per global store (KN_VEC_OUT) vs per-entry (_C_novec)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6vect
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tree.py tests/test_gpu.py > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
: > $O/ab.txt
for k in 16 50; do
  echo "== tree novec k=$k" >> $O/ab.txt
  AB_K=$k timeout -k 10 400 python scripts/ab_tree.py _novec 3 30 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { echo "AB_FAIL $k"; exit 1; }
done
cat $O/ab.txt
