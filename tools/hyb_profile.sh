#!/bin/bash
# PMC comparison of the config-2 expand kernel: T-table (default) vs the opt-in
# hybrid (DPF_EXPAND_HYBRID=1).  One counter group per rocprofv3 pass.
set -u
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/hybprof; mkdir -p $O
for mode in ttable hybrid; do
  [ $mode = hybrid ] && export DPF_EXPAND_HYBRID=1 || unset DPF_EXPAND_HYBRID
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$mode/trace -o trace --output-format csv -- python3 $R/tools/expand_once.py > /dev/null 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES -d $O/$mode/p1 -o p1 --output-format csv -- python3 $R/tools/expand_once.py > /dev/null 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR -d $O/$mode/p2 -o p2 --output-format csv -- python3 $R/tools/expand_once.py > /dev/null 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/$mode/p3 -o p3 --output-format csv -- python3 $R/tools/expand_once.py > /dev/null 2>&1 || exit 1
done
echo done
