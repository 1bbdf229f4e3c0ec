#!/bin/bash
# Getter copy-out A/B (900K K=16 host-to-host API): destination prefault on/off, interleaved
# over 6 repetitions on one box (host-side timings are noisy: medians of 7 iterations per run).
set -e
mkdir -p gpurun_out
out=gpurun_out/getter_ab.txt
: > $out
for rep in 1 2 3 4 5 6; do
  for pf in 1 0; do
    echo "== prefault $pf rep $rep" >> $out
    KN_COPY_PREFAULT=$pf timeout -k 10 60 ./bin/knn_cli --uniform 900000 --k 16 --api-bench 7 >> $out 2>&1
  done
done
for pf in 1 0 1 0; do
  echo "== K50 prefault $pf" >> $out
  KN_COPY_PREFAULT=$pf timeout -k 10 60 ./bin/knn_cli --uniform 900000 --k 50 --api-bench 5 >> $out 2>&1
done
