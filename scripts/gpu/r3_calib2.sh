#!/bin/bash
# Round 3: VALU issue-rate calibration, extended opcode set (csrc/tools/valu_rate.hip).
set -o pipefail
O=gpurun_out/calib
mkdir -p $O
timeout -k 10 200 ./bin/valu_rate 10000 > $O/valu_rate2.jsonl 2> $O/valu_rate2.err || { echo VALU_FAIL; cat $O/valu_rate2.err; exit 1; }
python3 -c "
import json
for l in open('$O/valu_rate2.jsonl'):
    r=json.loads(l); print('%-30s w=%d %.2f' % (r['op'], r['waves_per_simd'], r['simd_cycles_per_wave_inst']))
"
