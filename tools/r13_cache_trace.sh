#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of heavy hitters at 2^18
# clients with the expansion cache: gpurun_out/r13_cache_trace/hh_kernel_stats.csv
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r13_cache_trace -o hh --output-format csv -- python3 bench.py --workload heavy_hitters --no-cpu-baseline --keys-log 18 --steps 1 --warmup 0 > gpurun_out/r13_cache_trace.log 2>&1 || exit 1
head -6 gpurun_out/r13_cache_trace/hh_kernel_stats.csv
tail -1 gpurun_out/r13_cache_trace.log
