#!/bin/bash
# Expansion cache under memory pressure: the full-size heavy hitters test after
# the rest of the GPU suite's batch tests (torch's caching allocator holding
# their memory), then the 2^20 bench with and without the cache.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_batch_context_gpu.py tests/test_heavy_hitters_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 600 --timeout-method thread > gpurun_out/r13_oom_tests.log 2>&1 || { tail -30 gpurun_out/r13_oom_tests.log; exit 1; }
tail -1 gpurun_out/r13_oom_tests.log
hh() { timeout -k 10 400 python bench.py --workload heavy_hitters --no-cpu-baseline "$@" 2>>gpurun_out/r13_oom_hh.err | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(json.dumps({k: d.get(k) for k in ('value','seconds_per_pass','aes_blocks_per_s','verified')}), d['roofline']['frac'])"; }
echo "cache 2^20:"; hh || exit 1
