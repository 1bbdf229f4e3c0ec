#!/bin/bash
# Binning block size 256 vs 1024 (KN_BIN_THREADS) across configurations; two passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5bin
mkdir -p $O
: > $O/ab.txt
one() {  # label env -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" MASTER_PORT=$((29700 + RANDOM % 200)) timeout -k 10 200 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('ms_build'))" >> $O/ab.txt
}
for pass in 1 2; do
for T in 256 1024; do
  one "bin$T 20/5" KN_BIN_THREADS=$T -- --steps 20 --warmup 5
  one "bin$T 200/50" KN_BIN_THREADS=$T -- --steps 200 --warmup 50
  one "bin$T k32" KN_BIN_THREADS=$T -- --k 32 --steps 100 --warmup 30
  one "bin$T k50" KN_BIN_THREADS=$T -- --k 50 --steps 100 --warmup 30
  one "bin$T clustered" KN_BIN_THREADS=$T -- --gen clustered --steps 60 --warmup 20
  one "bin$T surface" KN_BIN_THREADS=$T -- --gen surface --steps 60 --warmup 20
  one "bin$T 10M k32" KN_BIN_THREADS=$T -- --n 10000000 --k 32 --steps 20 --warmup 10
  one "bin$T dist 200/50" KN_BIN_THREADS=$T -- --dist --steps 200 --warmup 50
  one "bin$T 300K" KN_BIN_THREADS=$T -- --n 300000 --steps 200 --warmup 50
done
done
sort $O/ab.txt
