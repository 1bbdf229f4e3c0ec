#!/bin/bash
# Round 3: PMC of the tree query kernel (900K clustered, K=16): wait vs VALU share.
set -o pipefail
export PYTHONPATH=$PWD
O=gpurun_out/treepmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-include-regex "knn_tree_kernel|knn_tile_kernel" -d $R/$O/p1 -o run -- python3 $R/scripts/diag_tree.py clustered 900000 16 > $R/$O/p1.log 2>&1 || { echo P1_FAIL; tail $R/$O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-include-regex "knn_tree_kernel|knn_tile_kernel" -d $R/$O/p2 -o run -- python3 $R/scripts/diag_tree.py clustered 900000 16 > $R/$O/p2.log 2>&1 || { echo P2_FAIL; tail $R/$O/p2.log; exit 1; }
ls -R $R/$O | head -30
