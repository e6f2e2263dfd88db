#!/bin/bash
# Collects the rocprofv3 evidence for bench.py's dominant kernel on one MI355X.
# Usage (on the GPU box, from the repo root): bash profiles/profile.sh <tag> [bench args]
# Kernel trace/stats and every PMC pass run as separate processes (PMC never
# combined with tracing); each pass is time-limited.
set -u
TAG=${1:-r01}; shift || true
ARGS=${@:-"--steps 5 --warmup 1 --no-cpu-baseline"}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() { # name, rocprof args...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $PWD/bench.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run trace --kernel-trace --stats || exit 1
run pmc_fetch --pmc FETCH_SIZE || exit 1
run pmc_write --pmc WRITE_SIZE GRBM_GUI_ACTIVE || exit 1
run pmc_sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES || exit 1
run pmc_sq2 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD || exit 1
echo done
