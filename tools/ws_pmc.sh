#!/bin/bash
# One PMC pass over tools/expand_ab.py --one for the wave-specialised and the
# octet expand kernels (config 2); per-dispatch counters land in gpurun_out/wspmc/.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/wspmc; mkdir -p $O
C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
DPF_EXPAND_WS=1 timeout -s KILL 120 rocprofv3 --pmc $C -d $O/ws -o ws --output-format csv -- python3 $R/tools/expand_ab.py --one --reps 2 > $O/ws.log 2>&1 || exit 1
DPF_EXPAND_WS=0 timeout -s KILL 120 rocprofv3 --pmc $C -d $O/oct -o oct --output-format csv -- python3 $R/tools/expand_ab.py --one --reps 2 > $O/oct.log 2>&1 || exit 1
echo ok
