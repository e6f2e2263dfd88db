#!/bin/bash
# First expansion level of both keys of a pair hashed together (pairl1,
# -DDPF_BATCH_PAIR_L1=1, ILP4) vs per key (base, ILP2): parity of pairl1, then
# heavy hitters 2^18 clients, two alternating rounds, with the probes noconv
# (no sampling divisions) and nostore (no expansion-cache stores).
set -u
mkdir -p gpurun_out
L=distributed_point_functions_amd/lib/libdpf_hip.so
cp $L vlib/_orig.so
cp vlib/pairl1.so $L
timeout -k 10 600 python -u -m pytest tests/test_batch_context_gpu.py tests/test_heavy_hitters_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r13_pairl1_tests.log 2>&1 || { cp vlib/_orig.so $L; tail -30 gpurun_out/r13_pairl1_tests.log; exit 1; }
tail -1 gpurun_out/r13_pairl1_tests.log
cp vlib/_orig.so $L
for r in 1 2; do
  bash tools/ab_lib.sh "--workload heavy_hitters --keys-log 18" base pairl1 || exit 1
  DPF_BENCH_SKIP_VERIFY=1 bash tools/ab_lib.sh "--workload heavy_hitters --keys-log 18" noconv nostore || exit 1
done
