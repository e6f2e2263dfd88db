#!/bin/bash
# Runs the wave-specialisation microbenchmark variants (tools/ws_microbench.hip).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out/ws
for b in "$@"; do
  timeout -k 10 120 $R/tools/wsmb_$b > $R/gpurun_out/ws/wsmb_$b.txt
  cat $R/gpurun_out/ws/wsmb_$b.txt
done
