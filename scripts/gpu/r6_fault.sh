#!/bin/bash
# Round 6: the id_map-gather fault of the vector-store re-rank, reproduced on the bounds-checked
# pre-fix build (_C_chkold: no fault, the violation is recorded), then the fixed release build on
# the test that faulted, then the whole GPU suite
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6fault
mkdir -p $O
KN_C_VARIANT=chkold timeout -k 10 120 python scripts/diag_idmap_vec.py > $O/chkold.txt 2>&1 || { echo CHK_FAIL; tail -20 $O/chkold.txt; exit 1; }
cat $O/chkold.txt | grep -v amdgpu.ids
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread "tests/test_gpu_distributed.py::test_device_plan_matches_host_plan" > $O/one.txt 2>&1 || { echo ONE_FAIL; tail -30 $O/one.txt; exit 1; }
tail -2 $O/one.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
