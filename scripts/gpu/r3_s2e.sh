#!/bin/bash
# Round 3 (session 2): packed outer rows A/B (_C vs _C_opack), host API with the block cache
# on / off (staging off).
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2e
mkdir -p $O
timeout -k 10 300 python scripts/ab_multi.py opack 900000 8,16,24,32,40 uniform 12 > $O/ab_opack.jsonl 2>> $O/err.log || { echo AB_FAIL; tail -20 $O/err.log; exit 1; }
timeout -k 10 300 python scripts/ab_multi.py opack 900000 16 blue,clustered 8 >> $O/ab_opack.jsonl 2>> $O/err.log || { echo AB2_FAIL; tail -20 $O/err.log; exit 1; }
timeout -k 10 300 python scripts/ab_multi.py opack 100000 8,16 uniform 12 >> $O/ab_opack.jsonl 2>> $O/err.log || { echo AB3_FAIL; tail -20 $O/err.log; exit 1; }
cat $O/ab_opack.jsonl
for c in 0 1; do
  KN_ARENA_CACHE=$c timeout -k 10 200 ./bin/knn_cli --uniform 900000 --k 16 --api-bench 7 > $O/api16_c$c.json 2> $O/api16_c$c.log || { echo API_FAIL; tail $O/api16_c$c.log; exit 1; }
  echo "cache=$c $(cat $O/api16_c$c.json)"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_tree.py -x -q --timeout 120 --timeout-method thread -k "pipelined or engine" > $O/pytest_pipe.log 2>&1 || { echo PIPE_TEST_FAIL; tail -30 $O/pytest_pipe.log; exit 1; }
tail -1 $O/pytest_pipe.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 > $O/bench_plain$r.json 2>> $O/err.log || { echo BENCH_FAIL; exit 1; }
  timeout -k 10 200 python bench.py --steps 50 --warmup 10 --pipeline > $O/bench_pipe$r.json 2>> $O/err.log || { echo BENCHP_FAIL; exit 1; }
  python - $O/bench_plain$r.json $O/bench_pipe$r.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f, d["ms_per_step"], d["value"], d["check"], d.get("pipelined"))
PY
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --k 50 --pipeline > $O/bench_pipe50.json 2>> $O/err.log && tail -c 400 $O/bench_pipe50.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_pipe -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --steps 30 --pipeline > $GRAFT_REPO_ROOT/$O/prof_pipe.log 2>&1) || { echo PROF_FAIL; exit 1; }
echo done
