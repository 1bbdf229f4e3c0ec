#!/bin/bash
# Rehearse the driver's multi-GPU launch on a 1-GPU box: N ranks (torchrun, one process per
# rank) all on cuda:0. RCCL refuses several ranks per GPU, so the collectives go through gloo
# with host staging (HostStagedTransport); everything else is the bench's multi-GPU code path.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD KN_SAME_DEVICE=1 KN_DIST_BACKEND=gloo
for N in 2 4 8; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $N --points 300000 --steps 3 --warmup 1 > gpurun_out/rehearse$N.json 2> gpurun_out/rehearse$N.err || { echo REHEARSE${N}_FAIL; grep -v "^\[bench" gpurun_out/rehearse$N.err | tail -15; exit 1; }
  echo "N=$N"; tail -1 gpurun_out/rehearse$N.json | cut -c1-700
done
