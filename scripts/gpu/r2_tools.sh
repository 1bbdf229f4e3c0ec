#!/bin/bash
# tools/profile.sh on the final tree: kernel stats + step timeline of the headline bench and the
# PMC passes of the K=16 query kernel.
set -o pipefail
bash tools/profile.sh timeline --steps 20 > gpurun_out/tools_timeline.txt 2>&1 || { echo TL_FAIL; tail gpurun_out/tools_timeline.txt; exit 1; }
tail -30 gpurun_out/tools_timeline.txt
bash tools/profile.sh pmc 16 900000 > gpurun_out/tools_pmc16.txt 2>&1 || { echo PMC_FAIL; tail gpurun_out/tools_pmc16.txt; exit 1; }
cat gpurun_out/tools_pmc16.txt
