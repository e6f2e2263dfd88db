#!/bin/bash
# Heavy hitters at 2^20 clients: batch-context GPU tests, then the bench with
# the lean kernel and with the general one (expansion-cache event counters in
# each line), then one pass under a kernel trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_batch_context_gpu.py tests/test_heavy_hitters_gpu.py -x -q --timeout 240 --timeout-method thread > gpurun_out/hhd_tests.log 2>&1 || { tail -20 gpurun_out/hhd_tests.log; exit 1; }
tail -1 gpurun_out/hhd_tests.log
for v in cur env:DPF_BATCH_GATHER=1; do
  e=""; [ $v = cur ] || e=${v#env:}
  f=gpurun_out/hhd_$(echo $v|tr ':=' '__').json
  env $e timeout -k 10 300 python bench.py --workload heavy_hitters --no-cpu-baseline --steps 2 > $f 2>gpurun_out/hhd.err || { tail gpurun_out/hhd.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$f'))
print('$v', d['seconds_per_pass'], d['roofline']['frac'], d['expansion_cache_events'], d['batch_context_device_bytes'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/hhd_trace -o hh --output-format csv -- python3 bench.py --workload heavy_hitters --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/hhd_trace.log 2>&1 || exit 1
cut -c1-160 gpurun_out/hhd_trace/hh_kernel_stats.csv | head -5
