#!/bin/bash
# Round 3 (session 2): world-1 steady step without routing passes, flag stored by the flag kernel, direct input
# inside the step graph; GPU suite, distributed vs native step, kernel stats of the dist step.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/s2n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
: > $O/dist.txt
for r in 1 2; do
  timeout -k 10 200 python bench.py --dist --steps 100 --warmup 10 > $O/_d.json 2>> $O/err.log || { echo DIST_FAIL; tail $O/err.log; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/_d.json') if l.startswith('{')][-1]); print('dist', round(d['ms_per_step'],4), '%.3e' % d['value'], d['check'], d.get('invalid_async_steps'), d.get('host_enqueue_ms_per_step'))" >> $O/dist.txt
  timeout -k 10 200 python bench.py --no-pipeline --steps 100 --warmup 10 --no-check > $O/_s.json 2>> $O/err.log || { echo SER_FAIL; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/_s.json') if l.startswith('{')][-1]); print('serial', round(d['ms_per_step'],4), '%.3e' % d['value'])" >> $O/dist.txt
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-check > $O/_p.json 2>> $O/err.log || { echo PIPE_FAIL; exit 1; }
  python -c "
import json; d=json.loads([l for l in open('$O/_p.json') if l.startswith('{')][-1]); print('pipelined', round(d['ms_per_step'],4), '%.3e' % d['value'])" >> $O/dist.txt
done
cat $O/dist.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/pdist -o run -- python3 $GRAFT_REPO_ROOT/bench.py --dist --steps 30 --warmup 5 --no-check > $GRAFT_REPO_ROOT/$O/pdist.log 2>&1) || { echo PROF_FAIL; tail $O/pdist.log; exit 1; }
echo done
