#!/bin/bash
# Start seeds of the next key pair loaded one pair ahead (pf,
# -DDPF_BATCH_PREFETCH=1) vs at use (nopf): heavy hitters 2^18 clients with the
# expansion cache, two alternating rounds; parity of pf first.
set -u
mkdir -p gpurun_out
L=distributed_point_functions_amd/lib/libdpf_hip.so
cp $L vlib/_orig.so
cp vlib/pf.so $L
timeout -k 10 600 python -u -m pytest tests/test_batch_context_gpu.py tests/test_heavy_hitters_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r13_pf_tests.log 2>&1 || { cp vlib/_orig.so $L; tail -30 gpurun_out/r13_pf_tests.log; exit 1; }
tail -1 gpurun_out/r13_pf_tests.log
cp vlib/_orig.so $L
for r in 1 2; do
  bash tools/ab_lib.sh "--workload heavy_hitters --keys-log 18" nopf pf || exit 1
done
