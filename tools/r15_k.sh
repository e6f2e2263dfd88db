#!/bin/bash
# r15 lease K: the small-tree launch for every leaf policy (parity, grid on/off
# for tuples and IntModN), and config 3's pipelined copy with 2 or 4 pieces.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
B=distributed_point_functions_amd/lib/dpf_benchmark
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_api_gpu.py tests/test_cpp_api_gpu.py \
  tests/test_reference_benchmarks_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r15k_tests.log 2>&1
rc=$?; tail -2 $O/r15k_tests.log; [ $rc -eq 0 ] || { tail -30 $O/r15k_tests.log; exit 1; }
F='EvaluateRegularDpf<(Tuple<uint32_t, uint32_t>|Tuple<uint32_t, uint64_t>|Tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>|Tuple<MyIntModN x5>|Tuple<MyIntModN64 x5>)>/(12|14|16)$'
for v in 1 0; do
  DPF_EXPAND_SMALL=$v timeout -k 10 300 $B "--benchmark_filter=$F" > $O/r15k_grid_s$v.txt 2>&1 || exit 1
  grep BM_ $O/r15k_grid_s$v.txt | awk -v v=$v '{print "small=" v, $1, $2}'
done
DPF_HOST_TIMING=1 timeout -k 10 120 $B '--benchmark_filter=EvaluateRegularDpf<Tuple<MyIntModN x5>>/12$' > $O/r15k_modn_timing.txt 2>&1 || exit 1
grep -h "BM_\|host timing" $O/r15k_modn_timing.txt
export DPF_HIP_D2H_PIPELINE=1
for mib in 16384 8192; do
  DPF_HIP_D2H_PIECE_MIB=$mib DPF_HIP_D2H_TRACE=1 timeout -k 10 500 python bench.py --workload full_domain_u128 --host-output \
    --host-output-reps 6 --no-cpu-baseline --steps 2 --warmup 1 > $O/r15k_u128_p$mib.json 2> $O/r15k_u128_p$mib.err \
    || { tail $O/r15k_u128_p$mib.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], [round(x) for x in d['api_level']['api_ms_per_call']])" $O/r15k_u128_p$mib.json piece$mib
  grep "_d2h\]" $O/r15k_u128_p$mib.err | tail -6
done
