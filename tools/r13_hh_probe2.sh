#!/bin/bash
# Heavy hitters (2^18 clients, expansion cache) cost probes: base vs no
# sampling divisions (noconv) vs no expansion-cache stores (nostore).  Probe
# outputs are wrong by construction: DPF_BENCH_SKIP_VERIFY=1.
set -u
mkdir -p gpurun_out
export DPF_BENCH_SKIP_VERIFY=1
for r in 1 2; do
  bash tools/ab_lib.sh "--workload heavy_hitters --keys-log 18" base noconv nostore || exit 1
done
