#!/bin/bash
# Large clouds: binning block threads x items (10M K=32, 12.5M K=16 dist share), two passes
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5big
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
  one "10M base" X=1 -- --n 10000000 --k 32 --steps 20 --warmup 10
  one "10M t256 i16384" KN_BIN_THREADS=256 KN_BIN_ITEMS=16384 -- --n 10000000 --k 32 --steps 20 --warmup 10
  one "10M t256 i65536" KN_BIN_THREADS=256 KN_BIN_ITEMS=65536 -- --n 10000000 --k 32 --steps 20 --warmup 10
  one "10M t1024 i16384" KN_BIN_THREADS=1024 KN_BIN_ITEMS=16384 -- --n 10000000 --k 32 --steps 20 --warmup 10
  one "12.5M dist base" X=1 -- --dist --n 12500000 --k 16 --steps 20 --warmup 5
  one "12.5M dist t256 i65536" KN_BIN_THREADS=256 KN_BIN_ITEMS=65536 -- --dist --n 12500000 --k 16 --steps 20 --warmup 5
  one "12.5M dist t1024 i16384" KN_BIN_THREADS=1024 KN_BIN_ITEMS=16384 -- --dist --n 12500000 --k 16 --steps 20 --warmup 5
done
sort $O/ab.txt
