#!/bin/bash
# Round 6: the capture crash. The standalone reproducer against torch's bundled
# HIP runtime (the extension's), then the engine's own unrolled two-query-stream capture with
# phase marks (last: a segfault ends the call by design)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r6c
mkdir -p $O
TL=$(python -c "import torch,os;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
H=/tmp/kn_torch_hip
mkdir -p $H && ln -sf $TL/libamdhip64.so $H/libamdhip64.so.7
for args in "4 1 0 5 2 0 2 1" "10 1 0 5 2 0 2 1" "4 1 0 5 2 0 1 0" "4 0 0 5 2 0 2 1"; do
  tag=$(echo $args | tr ' ' _)
  echo "repro (torch HIP) $args"
  LD_LIBRARY_PATH=$H:$TL timeout -k 10 60 ./bin/repro_capture $args > $O/repro_t_$tag.txt 2>&1
  rc=$?
  echo "rc $rc"; head -1 $O/repro_t_$tag.txt; tail -2 $O/repro_t_$tag.txt
  if [ $rc -ne 0 ]; then exit 0; fi
done
echo "engine unrolled with two query streams (marks)"
KN_PIPE_TRACE=1 KN_PIPE_UNROLL_QS2=1 KN_PIPE_SETS=2 KN_BENCH_SUPERVISE=0 timeout -k 10 120 python bench.py --steps 40 --warmup 10 --unroll 4 --no-check > $O/eng.json 2> $O/eng.err
rc=$?
echo "rc $rc"; grep -a "\[pipeline\]" $O/eng.err | tail -8
