#!/bin/bash
# C API: single-GPU reference flow, multi-device entry (RCCL with one device; device copies
# with 2/4/8 virtual ranks), and the CMake-built (torch-free) library's GPU ctests
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_capi.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_capi.log 2>&1 || { echo CAPI_FAIL; tail -40 gpurun_out/pytest_capi.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/pytest_capi.log | tail -12
timeout -k 10 600 ctest --test-dir build_cmake -L gpu --output-on-failure > gpurun_out/ctest_gpu.log 2>&1 || { echo CTEST_FAIL; tail -30 gpurun_out/ctest_gpu.log; exit 1; }
tail -5 gpurun_out/ctest_gpu.log
