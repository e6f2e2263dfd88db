#!/bin/bash
# IntModN32 sampling with the N >= 2^31 branch (no normalisation shifts, top
# quotient digit by compare) vs without: parity tests of the Mod32 paths, then
# heavy hitters (2^18 clients) and Tuple<IntModN32 x2> full domain A/B.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_batch_context_gpu.py tests/test_key_batch_gpu.py tests/test_heavy_hitters_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r13_norm_tests.log 2>&1 || { tail -30 gpurun_out/r13_norm_tests.log; exit 1; }
tail -2 gpurun_out/r13_norm_tests.log
for r in 1 2; do
  bash tools/ab_lib.sh "--workload heavy_hitters --keys-log 18" nonorm norm || exit 1
  bash tools/ab_lib.sh "--workload full_domain_tuple --tuple-type intmodn32x2 --steps 5 --warmup 1" nonorm norm || exit 1
done
