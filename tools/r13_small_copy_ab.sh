#!/bin/bash
# Small pageable copies through a page-locked buffer (post) vs hipMemcpy on
# the pageable memory (pre): the reference benchmark suite's small sizes.
set -u
mkdir -p gpurun_out
L=distributed_point_functions_amd/lib/libdpf_hip.so
cp $L vlib/_orig.so
for r in 1 2; do
  for v in pre post; do
    cp vlib/$v.so $L
    echo "== $v"
    timeout -k 10 300 distributed_point_functions_amd/lib/dpf_benchmark --benchmark_filter='BM_EvaluateRegularDpf<(uint8_t|uint64_t|uint128)>/(12|16|20)|BM_EvaluateHierarchicalFull<uint8_t>|BM_KeyGeneration' 2>/dev/null | grep -v "^Benchmark" || { cp vlib/_orig.so $L; exit 1; }
  done
done
cp vlib/_orig.so $L
