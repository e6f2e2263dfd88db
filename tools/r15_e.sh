#!/bin/bash
# r15 lease E: the lane-quad latency mode of small EvaluateAt launches --
# parity (the point tests, the API's EvaluateAt grids), then the reference's
# BM_BatchEvaluation with it on (default) and off (DPF_POINTS_QUAD=0).
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_key_batch_gpu.py tests/test_api_gpu.py tests/test_kernels_gpu.py \
  tests/test_dcf_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r15e_tests.log 2>&1
rc=$?; tail -2 $O/r15e_tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for q in 1 0; do
    DPF_POINTS_QUAD=$q timeout -k 10 120 distributed_point_functions_amd/lib/dpf_benchmark \
      --benchmark_filter='BatchEvaluation' > $O/r15e_be_q${q}_r$r.txt 2>&1 || exit 1
    echo "quad=$q"; grep BM_ $O/r15e_be_q${q}_r$r.txt
  done
done
