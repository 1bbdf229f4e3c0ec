#!/bin/bash
# distributed path: GPU tests (loopback / RCCL world 1), steady-state async steps, benches
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_dist.log 2>&1 || { echo TESTS_FAIL; tail -40 gpurun_out/pytest_gpu_dist.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_dist.log
O=gpurun_out/bench_dist.jsonl
: > $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> $O 2> gpurun_out/b1.err || { echo B1_FAIL; tail gpurun_out/b1.err; exit 1; }
timeout -k 10 300 python bench.py --dist --steps 20 --warmup 5 >> $O 2> gpurun_out/b2.err || { echo B2_FAIL; tail gpurun_out/b2.err; exit 1; }
timeout -k 10 300 python bench.py --dist --sync-steps --steps 20 --warmup 5 >> $O 2> gpurun_out/b3.err || { echo B3_FAIL; tail gpurun_out/b3.err; exit 1; }
timeout -k 10 600 python bench.py --loopback 8 --steps 5 --warmup 2 >> $O 2> gpurun_out/b4.err || { echo B4_FAIL; tail gpurun_out/b4.err; exit 1; }
timeout -k 10 600 python bench.py --loopback 8 --sync-steps --steps 5 --warmup 2 >> $O 2> gpurun_out/b5.err || { echo B5_FAIL; tail gpurun_out/b5.err; exit 1; }
python - <<'PY'
import json
for l in (x for x in open("gpurun_out/bench_dist.jsonl") if x.startswith("{")):
    d = json.loads(l)
    print(d["config"]["parallelism"], d.get("path"), round(d["ms_per_step"], 4), "ms", d.get("check"), d.get("stats", {}).get("n_halo"),
          d.get("steady_async"), d.get("invalid_async_steps"), d.get("n_halo_rank0"))
PY
