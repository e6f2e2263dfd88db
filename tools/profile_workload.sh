#!/bin/bash
# rocprofv3 evidence for one bench.py workload's dominant kernel: a kernel
# trace (--kernel-trace --stats) and four PMC passes, each its own process
# (PMC never combined with tracing) under its own time limit, then
# tools/pmc_summary.py -> gpurun_out/<tag>_<workload>_summary.json, tagged with
# the workload so bench.py quotes it for that workload only.
# Usage (GPU box, repo root):
#   bash tools/profile_workload.sh <tag> <workload tag> '<kernel substring>' launch:<warmup> -- <bench.py args>
#   bash tools/profile_workload.sh <tag> <workload tag> '<kernel substring>' total:<passes> -- <bench.py args>
# launch:W  per-launch averages over the timed launches (the first W skipped);
# total:P   sums over every launch of the run, divided by P (warmup + timed
#           passes of a multi-launch workload such as one heavy-hitters pass).
set -u
TAG=$1; WL=$2; KERNEL=$3; MODE=$4; shift 4
[ "${1:-}" = "--" ] && shift
ARGS="$*"
OUT=$PWD/gpurun_out/prof_${TAG}_${WL}
mkdir -p $OUT
export TMPDIR=/tmp
LIMIT=${PROFILE_PASS_LIMIT:-300}
run() { # name, rocprof args...
  local name=$1; shift
  timeout -k 10 $LIMIT rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $PWD/bench.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?; echo "$WL $name rc=$rc"; return $rc
}
run trace --kernel-trace --stats || exit 1
run pmc_fetch --pmc FETCH_SIZE || exit 1
run pmc_write --pmc WRITE_SIZE GRBM_GUI_ACTIVE || exit 1
run pmc_sq1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES || exit 1
run pmc_sq2 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD || exit 1
case $MODE in
  launch:*) SEL="--skip ${MODE#launch:}" ;;
  total:*) SEL="--total --passes ${MODE#total:}" ;;
  *) echo "bad mode $MODE"; exit 2 ;;
esac
python3 tools/pmc_summary.py $OUT "$KERNEL" --bench-log $OUT/trace.log --workload $WL --tag $TAG $SEL \
  > gpurun_out/${TAG}_${WL}_summary.json || exit 1
cp $OUT/trace/trace_kernel_stats.csv gpurun_out/${TAG}_${WL}_kernel_stats.csv
grep -E '"(avg_ns|gaes_per_s|effective_clock_ghz|lds_pipe_busy|valu_lane_ops_per_aes|hbm_traffic_bytes|write_amplification)"' gpurun_out/${TAG}_${WL}_summary.json
