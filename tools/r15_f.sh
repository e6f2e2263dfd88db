#!/bin/bash
# r15 lease F: DCF latency mode (dcf_fast_quad_kernel) parity, then the
# reference's BM_EvaluateDcf with it on (default) and off (DPF_DCF_QUAD=0).
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_dcf_gpu.py tests/test_host_api_cpu.py -x -q --timeout 300 \
  --timeout-method thread > $O/r15f_tests.log 2>&1
rc=$?; tail -2 $O/r15f_tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for q in 1 0; do
    DPF_DCF_QUAD=$q timeout -k 10 200 distributed_point_functions_amd/lib/dpf_benchmark \
      --benchmark_filter='EvaluateDcf<uint(64|128)' > $O/r15f_dcf_q${q}_r$r.txt 2>&1 || exit 1
    echo "quad=$q"; grep BM_ $O/r15f_dcf_q${q}_r$r.txt
  done
done
bash tools/ab.sh --tag r15f_dcf --rounds 1 -- "--workload dcf" cur || exit 1
g++ -O2 -pthread tools/value_init_probe.cc -o /tmp/value_init_probe || exit 1
timeout -k 10 200 /tmp/value_init_probe 32 3 > $O/r15f_value_init_probe.jsonl 2>&1 || exit 1
cat $O/r15f_value_init_probe.jsonl
