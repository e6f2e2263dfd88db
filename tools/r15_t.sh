#!/bin/bash
# r15 lease T: the point kernels' new cut-over (lane quads up to num_cus x 256
# points) -- the key-batch suite, then BM_BatchEvaluation.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_key_batch_gpu.py tests/test_api_gpu.py -x -q --timeout 300 \
  --timeout-method thread > $O/r15t_tests.log 2>&1
rc=$?; tail -2 $O/r15t_tests.log; [ $rc -eq 0 ] || { tail -30 $O/r15t_tests.log; exit 1; }
for r in 1 2; do
  timeout -k 10 200 distributed_point_functions_amd/lib/dpf_benchmark '--benchmark_filter=BM_BatchEvaluation' > $O/r15t_be_r$r.txt 2>&1 || exit 1
  grep BM_ $O/r15t_be_r$r.txt
done
