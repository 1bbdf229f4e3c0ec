#!/bin/bash
# Multi-process rehearsal of the driver's N>1 bench command on ONE GPU: torch.distributed.run
# with 2 and 4 ranks, gloo host-staged collectives (RCCL refuses several ranks on one device).
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/rehearse
mkdir -p $O
for n in 2 4; do
  KN_DIST_BACKEND=gloo KN_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2955$n bench.py --gpus $n --steps 10 --warmup 3 > $O/w$n.json 2> $O/w$n.err || { echo FAIL $n; tail -20 $O/w$n.err; exit 1; }
  grep '"metric"' $O/w$n.json | python -c "import sys,json;d=json.loads(sys.stdin.read());print('world', d['n_gpus'], round(d['ms_per_step'],3), d['check'], d['invalid_async_steps'], d['rank_grid'], d['n_halo_rank0'])"
done
