#!/bin/bash
# r15 lease N: small RESULTS written by the kernels straight into
# page-locked memory (PinnedOut, <= 1 MiB) -- parity, then
# on/off (DPF_OUTPUT_ZERO_COPY=0) over the small calls, two rounds.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
B=distributed_point_functions_amd/lib/dpf_benchmark
timeout -k 10 900 python -u -m pytest tests/test_api_gpu.py tests/test_cpp_api_gpu.py tests/test_dcf_gpu.py \
  tests/test_key_batch_gpu.py tests/test_reference_benchmarks_gpu.py tests/test_host_copies_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r15n_tests.log 2>&1
rc=$?; tail -2 $O/r15n_tests.log; [ $rc -eq 0 ] || { tail -30 $O/r15n_tests.log; exit 1; }
F='EvaluateRegularDpf<(uint8_t|uint64_t)>/(12|16)$|BM_EvaluateDcf<uint64_t>/(4|24)$|BM_BatchEvaluation<XorWrapper<uint128>>/100/4000|HierarchicalFull<uint64_t>/(1|15)$'
for r in 1 2; do
  for z in 1 0; do
    DPF_OUTPUT_ZERO_COPY=$z timeout -k 10 200 python bench.py --log-domain 20 --steps 500 --warmup 50 --no-cpu-baseline \
      > $O/r15n_c1_z${z}_r$r.json 2> $O/r15n_c1_z${z}_r$r.err || { tail $O/r15n_c1_z${z}_r$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'config1', round(d['ms_per_step']*1e3,1), 'us/step')" $O/r15n_c1_z${z}_r$r.json zc=$z
    DPF_OUTPUT_ZERO_COPY=$z timeout -k 10 300 $B "--benchmark_filter=$F" > $O/r15n_grid_z${z}_r$r.txt 2>&1 || exit 1
    grep BM_ $O/r15n_grid_z${z}_r$r.txt | sed -E 's/ +([0-9]+) ns.*/ \1/' | awk -v z=$z '{print "zc=" z, $0}'
  done
done
