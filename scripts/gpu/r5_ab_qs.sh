#!/bin/bash
# A/B: second query stream in the unrolled pipeline graphs (KN_PIPE_QSTREAMS=2), interleaved
# processes on one box, 200/50 and the driver's 20/5; rocprof timeline of each; then (last step,
# may crash) the joined-stream RCCL capture repro with native backtraces.
set -o pipefail
export PYTHONPATH=$PWD TMPDIR=/tmp
O=gpurun_out/${OUT_DIR:-r5qs}
mkdir -p $O
for rep in 1 2 3; do
  for qs in 1 2; do
    KN_PIPE_QSTREAMS=$qs timeout -k 10 120 python bench.py --steps 200 --warmup 50 --no-check > $O/b200_q${qs}_$rep.json 2> $O/b200_q${qs}_$rep.err || { echo BENCH_FAIL; tail $O/b200_q${qs}_$rep.err; exit 1; }
    KN_PIPE_QSTREAMS=$qs timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-check > $O/b20_q${qs}_$rep.json 2> $O/b20_q${qs}_$rep.err || { echo BENCH_FAIL; tail $O/b20_q${qs}_$rep.err; exit 1; }
  done
done
for f in $O/b*.json; do echo "$f $(python -c "import json;print(round(json.loads(open('$f').read().splitlines()[-1])['ms_per_step'],4))")"; done
for qs in 1 2; do
  (cd /tmp && KN_PIPE_QSTREAMS=$qs timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_q$qs -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-check --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof_q$qs.log 2>&1) || { echo PROF_FAIL; exit 1; }
done
echo "--- joined-stream capture repro (forced collectives, KN_DIST_CAPTURE_JOINED=1)"
KN_DIST_CAPTURE=1 KN_DIST_CAPTURE_JOINED=1 NCCL_DEBUG=INFO MASTER_PORT=29581 timeout -k 10 200 python -X faulthandler bench.py --dist --force-collectives --steps 20 --warmup 5 --no-check > $O/joined.json 2> $O/joined.err
echo "joined exit $?"
tail -5 $O/joined.err
echo done
