#!/bin/bash
# Rehearsal of the driver's N>1 bench invocation on one GPU: torch.distributed.run, 2 and 4
# processes sharing the GPU, gloo host-staged transport (RCCL refuses several ranks per GPU)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5rehearse
mkdir -p $O
for n in 2 4; do
KN_DIST_BACKEND=gloo KN_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29800 + n)) bench.py --gpus $n --steps 20 --warmup 5 > $O/n$n.log 2>&1 || { echo "REHEARSAL_FAIL n=$n"; tail -30 $O/n$n.log; exit 1; }
grep '^{' $O/n$n.log | cut -c1-300
done
