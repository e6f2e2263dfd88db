#!/bin/bash
# r15 lease U: results of >= 4 MiB that arrive through the staging buffers are
# value-initialised on a helper thread during the DMA (DPF_OVERLAP_GROW=1,
# default) vs chunk by chunk (=0): parity, then the mid-size reference rows.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
B=distributed_point_functions_amd/lib/dpf_benchmark
timeout -k 10 900 python -u -m pytest tests/test_api_gpu.py tests/test_cpp_api_gpu.py tests/test_host_copies_gpu.py \
  tests/test_reference_benchmarks_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r15u_tests.log 2>&1
rc=$?; tail -2 $O/r15u_tests.log; [ $rc -eq 0 ] || { tail -30 $O/r15u_tests.log; exit 1; }
F='EvaluateRegularDpf<(uint64_t|uint128|Tuple<uint32_t, uint32_t>|Tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>|XorWrapper<uint128>)>/(18|20|22)$'
for r in 1 2; do
  for v in 1 0; do
    DPF_OVERLAP_GROW=$v timeout -k 10 300 $B "--benchmark_filter=$F" > $O/r15u_grid_g${v}_r$r.txt 2>&1 || exit 1
  done
done
for v in 1 0; do
  echo "overlap=$v"
  paste -d'|' <(grep BM_ $O/r15u_grid_g${v}_r1.txt | sed -E 's/ +([0-9]+) ns.*/|\1/') <(grep BM_ $O/r15u_grid_g${v}_r2.txt | sed -E 's/.* ([0-9]+) ns.*/\1/')
done
