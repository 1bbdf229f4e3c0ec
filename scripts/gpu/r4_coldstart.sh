#!/bin/bash
# Round 4: where the driver's 20/5 bench loses time against 200/50.
set -o pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
O=$R/gpurun_out/r4cold
mkdir -p "$O"
export PYTHONPATH=$R TMPDIR=/tmp
cd "$R"
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-check > "$O/b20_$i.json" 2> "$O/b20_$i.err" || exit 1
  timeout -k 10 120 python3 bench.py --gpus 1 --steps 200 --warmup 50 --no-check > "$O/b200_$i.json" 2> "$O/b200_$i.err" || exit 1
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 \
  > "$O/prof.log" 2>&1 || { tail -5 "$O/prof.log"; exit 1; }
db=$(find "$O/trace" -name "*.db" | head -1)
python3 "$R/scripts/coldstart.py" "$db" > "$O/coldstart.txt"
cat "$O/coldstart.txt" | tail -40
for f in "$O"/b*.json; do echo "$f $(python3 -c "import json,sys; print(json.load(open('$f'))['ms_per_step'])")"; done
