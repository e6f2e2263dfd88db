#!/bin/bash
# r15 lease P (diagnostic): hh_level_kernel's time per call when its start
# seeds are compacted first (DPF_BATCH_CACHE_MODE=gather) vs read in place
# from scattered cache rows (default slot table), 2^20 clients, same box.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
for m in default gather; do
  if [ $m = gather ]; then export DPF_BATCH_CACHE_MODE=gather; else unset DPF_BATCH_CACHE_MODE; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r15p_$m -o hh -- \
    python3 bench.py --workload heavy_hitters --no-cpu-baseline > $O/r15p_$m.log 2>&1 || exit 1
  echo "mode=$m"; find $O/r15p_$m -name "*kernel_stats.csv" -exec cut -c1-160 {} \;
done
