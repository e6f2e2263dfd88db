#!/bin/bash
# Upper bound of hiding the Mod32 sampling in the batch kernel: the current
# library vs a probe build without the divisions (DPF_PROBE_NO_CONVERT), one
# 2^18-client heavy-hitters pass each, alternating twice; then the host-output
# microbenchmark (tools/host_output_microbench.cc).
set -u
mkdir -p gpurun_out
for r in 1 2; do
  DPF_BENCH_SKIP_VERIFY=1 bash tools/ab_lib.sh "--workload heavy_hitters --keys-log 18" cur noconv || exit 1
done
timeout -k 10 240 tools/host_output_microbench 33 > gpurun_out/host_out_mb.txt 2>&1 || { cat gpurun_out/host_out_mb.txt; exit 1; }
cat gpurun_out/host_out_mb.txt
