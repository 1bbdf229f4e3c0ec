#!/bin/bash
# Points per binning block (KN_BIN_ITEMS) beyond 16K and on small / large clouds (three sets)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5items2
mkdir -p $O
: > $O/ab.txt
one() {  # label env -- args
  local label=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-check "$@" > $O/line.json 2> $O/err.txt || { echo "FAIL $label"; tail $O/err.txt; exit 1; }
  python -c "import json; d=json.loads(open('$O/line.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d.get('ms_build'))" >> $O/ab.txt
}
for pass in 1 2; do
for I in 4096 16384 32768; do
  one "i$I 900K 20/5" KN_BIN_ITEMS=$I -- --steps 20 --warmup 5
  one "i$I 900K surface" KN_BIN_ITEMS=$I -- --gen surface --steps 60 --warmup 20
  one "i$I 300K" KN_BIN_ITEMS=$I -- --n 300000 --steps 200 --warmup 50
  one "i$I pts20K" KN_BIN_ITEMS=$I -- --xyz data/pts20K.xyz --k 8 --steps 200 --warmup 50
  one "i$I 10M k32" KN_BIN_ITEMS=$I -- --n 10000000 --k 32 --steps 20 --warmup 10
  one "i$I dist" KN_BIN_ITEMS=$I -- --dist --steps 200 --warmup 50
done
done
sort $O/ab.txt
