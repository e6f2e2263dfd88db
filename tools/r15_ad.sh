#!/bin/bash
# r15 lease AD: the prefix walk in two fused passes over the stored
# evaluations and the context grown from the zero page while the walk runs --
# parity (incremental API suites), then the host-phase split of the synthetic
# hierarchical benchmark and HierarchicalFull/15.
set -u
O=gpurun_out; mkdir -p $O
B=distributed_point_functions_amd/lib/dpf_benchmark
timeout -k 10 900 python -u -m pytest tests/test_api_gpu.py tests/test_cpp_api_gpu.py tests/test_reference_benchmarks_gpu.py \
  tests/test_host_copies_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r15ad_tests.log 2>&1
rc=$?; tail -2 $O/r15ad_tests.log; [ $rc -eq 0 ] || { tail -30 $O/r15ad_tests.log; exit 1; }
DPF_HOST_TIMING=1 timeout -k 10 120 $B "--benchmark_filter=HierarchicalFull<uint64_t>/15\$" > $O/r15ad_hf.txt 2>&1 || exit 1
grep -h "BM_\|host timing" $O/r15ad_hf.txt
DPF_HOST_TIMING=1 timeout -k 10 300 python bench.py --workload synthetic_hierarchical --domain 32 > $O/r15ad_syn32.json 2> $O/r15ad_syn32.err || exit 1
grep -h "host timing" $O/r15ad_syn32.err $O/r15ad_hf.txt
timeout -k 10 300 python bench.py --workload synthetic_hierarchical --domain 128 > $O/r15ad_syn128.json 2> $O/r15ad_syn128.err || exit 1
for f in syn32 syn128; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['unit'])" $O/r15ad_$f.json $f; done
