#!/bin/bash
# Reproduction attempt of round 4's RCCL capture segfault: world-1 distributed pipeline with its
# stages captured on the JOINED (main) stream, forced collectives, RCCL debug output; the bench
# installs the native crash handler (backtrace on SIGSEGV)
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/r5joined
mkdir -p $O
for q in 1; do
KN_DIST_QSTREAMS=$q KN_DIST_CAPTURE=1 KN_DIST_CAPTURE_JOINED=1 NCCL_DEBUG=INFO MASTER_PORT=2988$q timeout -k 10 180 python bench.py --dist --force-collectives --steps 40 --warmup 10 > $O/q$q.log 2>&1
echo "qstreams $q exit $?"
grep -E '^\{|crash|Segmentation|SIGSEGV|backtrace|frame|#[0-9]+ |lib.*\.so' $O/q$q.log | grep -v "NCCL INFO" | head -40 | cut -c1-250
done
