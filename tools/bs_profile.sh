#!/bin/bash
# PMC passes over the bitsliced microbenchmark (one counter group per pass).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/bsm
for B in bsm_w4 bsm_w4v; do
  timeout -k 10 60 $R/tools/$B > $R/gpurun_out/bsm/$B.txt
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/bsm/p1_$B -o p1 --output-format csv -- $R/tools/$B > /dev/null
  timeout -s KILL 60 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_SMEM -d $R/gpurun_out/bsm/p2_$B -o p2 --output-format csv -- $R/tools/$B > /dev/null
done
