#!/bin/bash
# PMC passes over one fbsm variant (GPU box): issue, waits, clock.
# Usage: bash tools/fbs_pmc.sh <binary> <tag>
B=$1; TAG=$2; O=$PWD/gpurun_out/fbspmc_$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES -d $O/p1 -o p1 --output-format csv -- $B > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $O/p2 -o p2 --output-format csv -- $B > $O/p2.log 2>&1 || exit 1
echo pmc ok
