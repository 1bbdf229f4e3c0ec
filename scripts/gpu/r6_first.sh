#!/bin/bash
# Round 6, first GPU call: CU-mask probe, GPU tests, default bench, driver-style 2-rank rehearsal
# through the supervisor, then the standalone capture reproducer (last: it may segfault the host
# process by design)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6first
mkdir -p $O
timeout -k 10 120 ./bin/cu_mask_probe > $O/cumask.txt 2>&1 || { echo "PROBE_FAIL"; tail $O/cumask.txt; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "PYTEST_FAIL"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo "BENCH_FAIL"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json | cut -c1-600
KN_DIST_BACKEND=gloo KN_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29811 bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2.log 2>&1 || { echo "REHEARSAL_FAIL"; tail -30 $O/n2.log; exit 1; }
grep '^{' $O/n2.log | cut -c1-400
for args in "4 1 0" "4 0 0" "2 1 0" "4 1 1" "10 0 0"; do
  echo "repro $args"
  timeout -k 10 60 ./bin/repro_capture $args > $O/repro_$(echo $args | tr ' ' _).txt 2>&1
  rc=$?
  echo "rc $rc"; tail -3 $O/repro_$(echo $args | tr ' ' _).txt
  if [ $rc -ne 0 ]; then break; fi
done
