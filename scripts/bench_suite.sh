#!/bin/bash
# Every BASELINE.json configuration on one MI355X (run through gpurun from the repo root).
# The headline runs at the driver's 20 timed / 5 warmup steps and at 200 / 50 (the GPU's steady
# clocks: from idle the query kernel takes 304-320 us for its first ~20 steps vs 291 us warm,
# profiles/r4_coldstart.txt); the other rows time 100-200 steps.
# One JSON line per configuration -> gpurun_out/bench_suite.jsonl (copy to profiles/).
#   1. pts20K.xyz, k=8, CPU kd-tree path            (+ the same file on the GPU)
#   2. 300K uniform, k=16, 1 GPU                     (pts300K.xyz is missing from the reference)
#   3. 900K blue-noise stand-in, k=16, 1 GPU         (900k_blue_cube.xyz is missing)
#      + the headline 900K uniform k=16 and the reference default k=50
#   4. 10M uniform, k=32, 1 GPU
#   5. 100M uniform, k=16, 8-way spatial split: the per-rank share (12.5M) through the RCCL
#      path at world 1, and all 8 ranks as loopback virtual ranks on the one GPU
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH=$PWD
OUT=gpurun_out/bench_suite.jsonl
ERR=gpurun_out/bench_suite.err
: > $OUT
: > $ERR
run() {  # run <timeout> <label> <bench args...>
  local t=$1 label=$2
  shift 2
  echo "== $label: $*" >> $ERR
  MASTER_PORT=$((29600 + RANDOM % 300)) timeout -k 10 $t python bench.py "$@" > gpurun_out/_line.json 2>> $ERR || { echo "FAIL $label"; tail -20 $ERR; exit 1; }
  python - "$label" >> $OUT <<'PY'
import json, sys
line = [l for l in open("gpurun_out/_line.json") if l.startswith("{")][-1]
d = json.loads(line)
d["suite_label"] = sys.argv[1]
print(json.dumps(d))
PY
  echo "ok $label"
}
run 200 "cfg1 pts20K k8 cpu-kdtree" --cpu-oracle --k 8 --steps 5
run 200 "cfg1b pts20K k8 gpu" --xyz data/pts20K.xyz --k 8 --steps 200 --warmup 50
run 200 "cfg2 300K uniform k16 gpu" --n 300000 --k 16 --steps 200 --warmup 50
run 200 "cfg3 900K blue k16 gpu" --gen blue --n 900000 --k 16 --steps 200 --warmup 50
run 200 "headline 900K uniform k16 gpu, driver 20/5" --n 900000 --k 16 --steps 20 --warmup 5
run 200 "headline 900K uniform k16 gpu, 200/50" --n 900000 --k 16 --steps 200 --warmup 50
run 200 "900K uniform k16 gpu, stream of 4 distinct clouds" --n 900000 --k 16 --steps 200 --warmup 50 --stream-clouds 4
run 200 "900K uniform k16 rccl world1 (native distributed pipeline)" --dist --n 900000 --k 16 --steps 200 --warmup 50
run 200 "900K uniform k16 rccl world1, forced collectives" --dist --force-collectives --n 900000 --k 16 --steps 200 --warmup 50
run 200 "900K uniform k50 gpu (reference K)" --n 900000 --k 50 --steps 100 --warmup 30
run 200 "900K uniform k50 gpu, driver 20/5" --n 900000 --k 50 --steps 20 --warmup 5
run 200 "900K uniform k64 gpu" --n 900000 --k 64 --steps 100 --warmup 30
run 300 "cfg4 10M uniform k32 gpu" --n 10000000 --k 32 --steps 20 --warmup 5
run 200 "900K points on surfaces k16 gpu (occupancy-adaptive grid)" --gen surface --n 900000 --k 16 --steps 100 --warmup 20
run 300 "900K clustered k16 gpu (occupancy-adaptive grid)" --gen clustered --n 900000 --k 16 --steps 100 --warmup 20
run 300 "cfg5a 12.5M/rank k16 rccl world1 (100M/8 share)" --dist --n 12500000 --k 16 --steps 20 --warmup 5
run 600 "cfg5b 100M k16 loopback 8 ranks on 1 gpu" --loopback 8 --n 12500000 --k 16 --steps 5 --warmup 2
cat $OUT
