#!/bin/bash
# r15 lease D: Mod32Leaf parks the half-octet's second leaf pair in scratch
# during the first value-hash group (vlib/park1.so = in-tree) vs not
# (vlib/park0.so, -DDPF_MOD32_PARK=0): kernel parity first, then the
# Tuple<IntModN32 x2> full-domain A/B on one box.
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_api_gpu.py -x -q \
  --timeout 300 --timeout-method thread > $O/r15d_tests.log 2>&1
rc=$?; tail -2 $O/r15d_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab.sh --tag r15d_tup --rounds 3 -- "--workload full_domain_tuple" lib:park1 lib:park0 || exit 1
# Small EvaluateAt calls are latency-bound (one wave per CU): does dropping
# the per-round s_load (lane-resident keys, vlib/rk1.so) shorten the chain?
L=distributed_point_functions_amd/lib/libdpf_hip.so
cp $L $O/.d_orig.so
for v in cur rk1 cur rk1; do
  [ $v = rk1 ] && cp vlib/rk1.so $L
  timeout -k 10 120 distributed_point_functions_amd/lib/dpf_benchmark \
    --benchmark_filter='BatchEvaluation.*/(10/40000|100/4000)$' > $O/r15d_be_$v.txt 2>&1
  rc=$?; cp $O/.d_orig.so $L; [ $rc -eq 0 ] || exit 1
  echo $v; grep BM_ $O/r15d_be_$v.txt
done
