#!/bin/bash
# Round 6, second call: changed-area GPU tests, CU-mask probe v2, baseline query PMC at K=16,
# capture reproducer against torch's HIP runtime, then the engine's own unrolled two-query-stream
# capture (last: a host segfault in the runtime ends the call by design)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 120 ./bin/cu_mask_probe > $O/cumask.txt 2>&1 || { echo "PROBE_FAIL"; tail $O/cumask.txt; }
awk 'NR>1{print $12, $14}' $O/cumask.txt | sort | uniq -c
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_tree.py -x -q --timeout 300 --timeout-method thread -k "loopback_layouts or unrolled or stream_batch or supervised" > $O/pytest.log 2>&1 || { echo "PYTEST_FAIL"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/profile.sh pmc 16 900000 > $O/pmc_k16.txt 2>&1 || { echo "PMC_FAIL"; tail $O/pmc_k16.txt; exit 1; }
grep -E "per wave|WAIT_ANY /|VALU /|conflict" $O/pmc_k16.txt
TL=$(python -c "import torch,os;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
for args in "4 1 0 5 2 0 2" "10 1 0 5 2 0 2" "4 1 1 5 2 0 2"; do
  tag=$(echo $args | tr ' ' _)
  echo "repro (torch HIP) $args"
  LD_LIBRARY_PATH=$TL timeout -k 10 60 ./bin/repro_capture $args > $O/repro_t_$tag.txt 2>&1
  rc=$?
  echo "rc $rc"; head -1 $O/repro_t_$tag.txt; tail -2 $O/repro_t_$tag.txt
  if [ $rc -ne 0 ]; then exit 0; fi
done
for sets in 2; do
  echo "engine unrolled with two query streams, sets $sets"
  KN_PIPE_UNROLL_QS2=1 KN_PIPE_SETS=$sets KN_BENCH_SUPERVISE=0 timeout -k 10 120 python bench.py --steps 40 --warmup 10 --unroll 4 > $O/eng_qs2_s$sets.json 2> $O/eng_qs2_s$sets.err
  rc=$?
  echo "rc $rc"; tail -c 400 $O/eng_qs2_s$sets.json; grep -a -m3 "signal\|libamdhip" $O/eng_qs2_s$sets.err
  if [ $rc -ne 0 ]; then exit 0; fi
done
