#!/bin/bash
# exact kernel: ball-cut rows + 1024-WG fallback grid (_C) vs 256-WG grid (_C_eg256); tests; benches
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_exact2.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/pytest_gpu_exact2.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_exact2.log
O=gpurun_out/ab_exact2.log
: > $O
for kh in "16 0" "50 0" "64 0"; do
  set -- $kh
  echo "== uniform k=$1 halo=$2" >> $O
  timeout -k 10 120 python scripts/ab_plan.py eg256 900000 $1 $2 10 >> $O 2>&1 || { echo AB_FAIL $kh; tail -5 $O; exit 1; }
done
echo "== clustered k=16" >> $O
timeout -k 10 300 python scripts/ab_plan.py eg256 900000 16 0 3 clustered >> $O 2>&1 || { echo AB_FAIL clustered; tail -5 $O; exit 1; }
grep -v amdgpu.ids $O
for a in "--k 16" "--k 50" "--k 64" "--gen clustered --k 16"; do
  timeout -k 10 300 python bench.py $a --steps 10 --warmup 3 2> gpurun_out/b.err | tee -a gpurun_out/bench_exact2.jsonl | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$a', round(d['ms_per_step'],4), 'ms', d.get('exact_path_queries'), d['check'])" || { echo BENCH_FAIL $a; tail gpurun_out/b.err; exit 1; }
done
