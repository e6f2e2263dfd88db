#!/bin/bash
# Table fill with batched T0 loads (fill) vs one dependent load per store
# (pre): small EvaluateUntil latency (reference suite) and the config-2 step.
set -u
mkdir -p gpurun_out
L=distributed_point_functions_amd/lib/libdpf_hip.so
cp $L vlib/_orig.so
for r in 1 2; do
  for v in pre fill; do
    cp vlib/$v.so $L
    echo "== $v"
    timeout -k 10 300 distributed_point_functions_amd/lib/dpf_benchmark --benchmark_filter='BM_EvaluateRegularDpf<(uint8_t|uint64_t)>/(12|14|16|18|20)|BM_EvaluateHierarchicalFull<uint8_t>/(1|7|15)$|BM_BatchEvaluation' 2>/dev/null | grep -v "^Benchmark" || { cp vlib/_orig.so $L; exit 1; }
  done
  bash tools/ab_lib.sh "--steps 10 --warmup 2" pre fill || { cp vlib/_orig.so $L; exit 1; }
done
cp vlib/_orig.so $L
