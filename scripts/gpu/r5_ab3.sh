#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5ab3
mkdir -p $O
for k in 16 50 32 8; do
  for v in slow sq0 ce0 rrun; do
    echo "k=$k $v: $(timeout -k 10 120 python scripts/ab_variant.py $v 900000 $k 20 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')"
  done
done | tee $O/ab.txt
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 50 --no-check > $O/res_$rep.json 2> $O/res_$rep.err || exit 1
  timeout -k 10 200 python bench.py --stream-clouds 4 --steps 200 --warmup 50 > $O/sc_$rep.json 2> $O/sc_$rep.err || exit 1
done
for f in $O/sc_*.json $O/res_*.json; do echo "$f $(python -c "import json;d=json.loads(open('$f').read().splitlines()[-1]);print(round(d['ms_per_step'],4), d.get('check'))")"; done
timeout -k 10 400 python -u -m pytest tests/test_gpu_tree.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for g in clustered surface; do
  timeout -k 10 200 python bench.py --gen $g --steps 100 --warmup 30 > $O/tree_$g.json 2> $O/tree_$g.err || { echo TREE_FAIL; tail $O/tree_$g.err; exit 1; }
  echo "$g $(python -c "import json;d=json.loads(open('$O/tree_$g.json').read().splitlines()[-1]);print(round(d['ms_per_step'],4), d.get('check'), d.get('exact_path_queries'))")"
done
