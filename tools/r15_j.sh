#!/bin/bash
# r15 lease J: quad rounds with the lookups first (DPF_QUAD_LOOKUP_FIRST=1,
# in-tree) vs state permuted first (vlib/qf0.so) on every latency-mode path;
# config 3's host copy phases (whole registration vs pipelined).
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
L=distributed_point_functions_amd/lib/libdpf_hip.so
B=distributed_point_functions_amd/lib/dpf_benchmark
cp $L $O/.j_orig.so
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_key_batch_gpu.py tests/test_dcf_gpu.py \
  -x -q --timeout 300 --timeout-method thread -k "small or quad or latency or dcf" > $O/r15j_tests.log 2>&1
rc=$?; tail -2 $O/r15j_tests.log; [ $rc -eq 0 ] || { tail -30 $O/r15j_tests.log; exit 1; }
F='BM_EvaluateDcf<uint64_t>/(4|12|24)$|BM_BatchEvaluation<XorWrapper<uint128>>/100/4000|EvaluateRegularDpf<(uint8_t|uint64_t)>/(12|16)$'
for r in 1 2; do
  for v in cur qf0; do
    if [ $v = qf0 ]; then cp vlib/qf0.so $L; else cp $O/.j_orig.so $L; fi
    timeout -k 10 200 python bench.py --log-domain 20 --steps 500 --warmup 50 --no-cpu-baseline \
      > $O/r15j_c1_${v}_r$r.json 2> $O/r15j_c1_${v}_r$r.err || { cp $O/.j_orig.so $L; tail $O/r15j_c1_${v}_r$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'config1', round(d['ms_per_step']*1e3,1), 'us/step', round(d['roofline']['launch_ms']*1e3,1), 'us launch')" $O/r15j_c1_${v}_r$r.json $v
    timeout -k 10 300 $B "--benchmark_filter=$F" > $O/r15j_grid_${v}_r$r.txt 2>&1 || { cp $O/.j_orig.so $L; exit 1; }
    grep BM_ $O/r15j_grid_${v}_r$r.txt | awk -v v=$v '{print v, $1, $2}'
  done
done
cp $O/.j_orig.so $L
for mode in default pipe; do
  if [ $mode = pipe ]; then export DPF_HIP_D2H_PIPELINE=1; else unset DPF_HIP_D2H_PIPELINE; fi
  DPF_HIP_D2H_TRACE=1 timeout -k 10 500 python bench.py --workload full_domain_u128 --host-output --host-output-reps 6 \
    --no-cpu-baseline --steps 2 --warmup 1 > $O/r15j_u128_$mode.json 2> $O/r15j_u128_$mode.err || { tail $O/r15j_u128_$mode.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], [round(x) for x in d['api_level']['api_ms_per_call']])" $O/r15j_u128_$mode.json $mode
  grep "_d2h\]" $O/r15j_u128_$mode.err | tail -6
done
