#!/bin/bash
# r15 lease G: host result vectors value-initialised by memmove from the zero
# page (GrowZeroed) -- the probe, the host-output parity tests, config 3's
# API-level line over 5 calls, config 2's; and config 1
# (log 20, the reference's CPU-runnable case) as a bench line.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
g++ -O2 -pthread tools/value_init_probe.cc -o /tmp/value_init_probe || exit 1
timeout -k 10 200 /tmp/value_init_probe 32 3 > $O/r15g_value_init_probe.jsonl 2>&1 || exit 1
cat $O/r15g_value_init_probe.jsonl
timeout -k 10 600 python -u -m pytest tests/test_api_gpu.py tests/test_host_copies_gpu.py tests/test_cpp_api_gpu.py \
  -x -q --timeout 300 --timeout-method thread > $O/r15g_tests.log 2>&1
rc=$?; tail -2 $O/r15g_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python bench.py --workload full_domain_u128 --host-output --host-output-reps 5 --no-cpu-baseline \
  --steps 3 --warmup 1 > $O/r15g_api_u128.json 2> $O/r15g_api_u128.err || { tail -20 $O/r15g_api_u128.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/r15g_api_u128.json')); print('u128', d['api_level']['api_ms_per_call'])"
timeout -k 10 300 python bench.py --host-output --host-output-reps 5 --no-cpu-baseline --steps 5 --warmup 1 \
  > $O/r15g_api_u64.json 2> $O/r15g_api_u64.err || { tail -20 $O/r15g_api_u64.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/r15g_api_u64.json')); print('u64', d['api_level']['api_ms_per_call'])"
timeout -k 10 300 python bench.py --log-domain 20 --steps 200 --warmup 20 > $O/r15g_config1.json 2> $O/r15g_config1.err \
  || { tail -20 $O/r15g_config1.err; exit 1; }
cat $O/r15g_config1.json
timeout -k 10 300 distributed_point_functions_amd/lib/dpf_benchmark '--benchmark_filter=EvaluateRegularDpf<(uint128|uint64_t)>' \
  > $O/r15g_grid_int.txt 2>&1 || exit 1
grep BM_ $O/r15g_grid_int.txt
