#!/bin/bash
# Stream priority A/B: engine build stream (KN_PIPE_PRIO 0 / 1 greatest / 2 least), second query
# stream (KN_PIPE_AUXPRIO), distributed build stream (KN_DIST_SIDE_PRIO); 900K K=16 200 / 50 and
# K=50, two interleaved passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5prio
mkdir -p $O
: > $O/ab.txt
python -c "
import torch, ctypes
torch.cuda.init()
lib = ctypes.CDLL('libamdhip64.so')
lo, hi = ctypes.c_int(), ctypes.c_int()
print('priority range least/greatest', lib.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi)), lo.value, hi.value)
" >> $O/ab.txt 2>&1
one() {  # label args...
  local label=$1; shift
  MASTER_PORT=$((29700 + RANDOM % 200)) timeout -k 10 120 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4))" >> $O/ab.txt
}
for pass in 1 2; do
  one "engine prio0" --steps 200 --warmup 50
  KN_PIPE_PRIO=1 one "engine prio1" --steps 200 --warmup 50
  KN_PIPE_PRIO=2 one "engine prio2" --steps 200 --warmup 50
  KN_PIPE_AUXPRIO=1 one "engine auxprio1" --steps 200 --warmup 50
  KN_PIPE_PRIO=2 KN_PIPE_AUXPRIO=1 one "engine prio2 auxprio1" --steps 200 --warmup 50
  KN_PIPE_QSTREAMS=1 KN_PIPE_PRIO=2 one "engine qs1 prio2" --steps 200 --warmup 50
  KN_PIPE_QSTREAMS=1 one "engine qs1 prio0" --steps 200 --warmup 50
  one "dist sprio0" --dist --steps 200 --warmup 50
  KN_DIST_SIDE_PRIO=1 one "dist sprio1" --dist --steps 200 --warmup 50
  KN_DIST_SIDE_PRIO=2 one "dist sprio2" --dist --steps 200 --warmup 50
  one "k50 prio0" --k 50 --steps 100 --warmup 30
  KN_PIPE_PRIO=2 one "k50 prio2" --k 50 --steps 100 --warmup 30
done
sort $O/ab.txt
