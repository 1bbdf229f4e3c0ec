#!/bin/bash
# tools/profile.sh -- rocprofv3 entry point for the kNN engine on MI355X (SURVEY §5 tracing).
#
#   tools/profile.sh kstats   [bench.py args]   per-kernel device time of the bench step
#   tools/profile.sh timeline [bench.py args]   kstats + the dispatches of the last step (gaps)
#   tools/profile.sh pmc K N                     counter passes on the query kernel (N points, K)
#
# Output: gpurun_out/profile/<mode>_<stamp>/ (rocpd sqlite) + summary.txt. Every rocprofv3 run has
# its own time limit; counter passes stay within one pass's hardware limits (<= 8 SQ, <= 4 TCC
# counters; FETCH_SIZE alone) and are collected with --kernel-trace only (no API tracing).
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
mode=${1:-kstats}
shift || true
stamp=$(date +%Y%m%d_%H%M%S)
O=$R/gpurun_out/profile/${mode}_$stamp
mkdir -p "$O"
# KN_BENCH_SUPERVISE=0: bench.py runs its job in-process (no child forked from a process the
# profiler's preload has already attached to the GPU)
export PYTHONPATH=$R TMPDIR=/tmp KN_BENCH_SUPERVISE=0
cd /tmp
case $mode in
  kstats|timeline)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run -- python3 "$R/bench.py" --no-check "$@" \
      > "$O/run.log" 2>&1 || { echo "rocprofv3 failed ($O/run.log)"; tail -5 "$O/run.log"; exit 1; }
    db=$(find "$O/trace" -name "*.db" | head -1)
    if [ "$mode" = timeline ]; then
      python3 "$R/scripts/prof_db.py" "$db" --timeline 24 > "$O/summary.txt"
    else
      python3 "$R/scripts/prof_db.py" "$db" > "$O/summary.txt"
    fi
    ;;
  pmc)
    K=${1:-16}
    N=${2:-900000}
    P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
    P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH"
    P3="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32"
    P4="FETCH_SIZE"
    P5="TCC_HIT_sum TCC_MISS_sum"
    i=0
    dbs=()
    for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
      i=$((i + 1))
      timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d "$O/p$i" -o run -- python3 "$R/scripts/prof_query.py" "$N" "$K" 2 \
        > "$O/p$i.log" 2>&1 || { echo "pmc pass $i failed ($O/p$i.log)"; tail -5 "$O/p$i.log"; exit 1; }
      dbs+=("$(find "$O/p$i" -name "*.db" | head -1)")
    done
    python3 "$R/scripts/pmc_summary.py" knn_tile_kernel "${dbs[@]}" > "$O/summary.txt"
    ;;
  *)
    echo "usage: tools/profile.sh kstats|timeline [bench.py args] | pmc K N"; exit 2 ;;
esac
cat "$O/summary.txt"
echo "summary: $O/summary.txt"
