#!/bin/bash
# Expansion cache of the batched incremental evaluation: parity (batch context,
# key batch, heavy hitters tests), then heavy hitters with and without it
# (DPF_BATCH_NO_CACHE=1), two alternating rounds at 2^18 clients, one at 2^20,
# then a kernel trace of the cached run at 2^18 (gpurun_out/r13_cache_trace).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_batch_context_gpu.py tests/test_key_batch_gpu.py tests/test_heavy_hitters_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r13_cache_tests.log 2>&1 || { tail -30 gpurun_out/r13_cache_tests.log; exit 1; }
tail -2 gpurun_out/r13_cache_tests.log
hh() { timeout -k 10 400 python bench.py --workload heavy_hitters --no-cpu-baseline "$@" 2>>gpurun_out/r13_cache_hh.err | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(json.dumps({k: d.get(k) for k in ('value','seconds_per_pass','aes_blocks_per_s','verified')}), d['roofline']['frac'])"; }
for r in 1 2; do
  echo "cache:";    hh --keys-log 18 || exit 1
  echo "no cache:"; DPF_BATCH_NO_CACHE=1 hh --keys-log 18 || exit 1
done
echo "cache 2^20:"; hh || exit 1
echo "no cache 2^20:"; DPF_BATCH_NO_CACHE=1 hh || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r13_cache_trace -o hh --output-format csv -- python3 bench.py --workload heavy_hitters --no-cpu-baseline --keys-log 18 --steps 1 --warmup 0 > gpurun_out/r13_cache_trace.log 2>&1 || exit 1
find gpurun_out/r13_cache_trace -name "*kernel_stats.csv" | head -1 | xargs head -8
