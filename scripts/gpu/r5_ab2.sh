#!/bin/bash
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5ab2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_tree.py tests/test_capi.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for k in 16 50 8 32; do
  for v in slow rrun; do
    echo "k=$k $v: $(timeout -k 10 120 python scripts/ab_variant.py $v 900000 $k 20 2>&1 | grep -v amdgpu.ids | tr '\n' ' ')"
  done
done | tee $O/ab.txt
for rep in 1 2; do
  for mode in batch step; do
    timeout -k 10 200 python bench.py --stream-clouds 4 --stream-mode $mode --steps 200 --warmup 50 > $O/sc_${mode}_$rep.json 2> $O/sc_${mode}_$rep.err || { echo SC_FAIL; tail $O/sc_${mode}_$rep.err; exit 1; }
  done
  timeout -k 10 200 python bench.py --steps 200 --warmup 50 --no-check > $O/res_$rep.json 2> $O/res_$rep.err || exit 1
done
for f in $O/sc_*.json $O/res_*.json; do echo "$f $(python -c "import json;d=json.loads(open('$f').read().splitlines()[-1]);print(round(d['ms_per_step'],4), d.get('check'))")"; done
for g in clustered surface; do
  timeout -k 10 200 python bench.py --gen $g --steps 100 --warmup 30 > $O/tree_$g.json 2> $O/tree_$g.err || { echo TREE_FAIL; tail $O/tree_$g.err; exit 1; }
  echo "$g $(python -c "import json;d=json.loads(open('$O/tree_$g.json').read().splitlines()[-1]);print(round(d['ms_per_step'],4), d.get('check'), d.get('exact_path_queries'))")"
done
bash scripts/gpu/r5_qs_dbg.sh
