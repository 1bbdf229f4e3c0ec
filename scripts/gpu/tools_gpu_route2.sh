#!/bin/bash
# Self-last routing (route_begin + route_unpack_split): distributed GPU tests, the RCCL world-1
# bench (before/after numbers), a timeline of one distributed step, and the 2/4-rank rehearsal.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > gpurun_out/route2_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/route2_tests.log; exit 1; }
tail -2 gpurun_out/route2_tests.log
timeout -k 10 200 python bench.py --dist --n 900000 --k 16 --steps 50 --warmup 10 > gpurun_out/route2_dist1.json 2> gpurun_out/route2_dist1.err || { echo DIST_FAIL; tail -20 gpurun_out/route2_dist1.err; exit 1; }
tail -1 gpurun_out/route2_dist1.json | cut -c1-400
timeout -k 10 200 python bench.py --n 900000 --k 16 --steps 50 --warmup 10 > gpurun_out/route2_native.json 2>/dev/null || { echo NATIVE_FAIL; exit 1; }
tail -1 gpurun_out/route2_native.json | cut -c1-300
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/route2_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --no-check --n 900000 --k 16 --steps 6 --warmup 2 > /dev/null 2>&1 || { echo PROF_FAIL; exit 1; }
cd $GRAFT_REPO_ROOT
python scripts/prof_timeline.py $(find gpurun_out/route2_prof -name "*.db" | head -1) meta_bbox 40 > gpurun_out/route2_timeline.txt 2>&1 || true
tail -40 gpurun_out/route2_timeline.txt
export KN_SAME_DEVICE=1 KN_DIST_BACKEND=gloo
for N in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $N --points 300000 --steps 3 --warmup 1 > gpurun_out/route2_rehearse$N.json 2> gpurun_out/route2_rehearse$N.err || { echo REHEARSE${N}_FAIL; grep -v "^\[bench" gpurun_out/route2_rehearse$N.err | tail -15; exit 1; }
  echo "N=$N"; tail -1 gpurun_out/route2_rehearse$N.json | cut -c1-500
done
