#!/bin/bash
# r14: EvaluateAt with four path chains per lane (eval_points4_kernel, the
# default where a launch fills the chip) vs two (DPF_POINTS_ILP=2).  Parity
# first (every point-evaluation test), then the bench A/B.
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_key_batch_gpu.py tests/test_fullsize_gpu.py::test_config4_batched_points_reconstruct_hit_counts tests/test_fullsize_gpu.py::test_config4_per_key_outputs_full_size -x -q --timeout 300 --timeout-method thread > $O/r14ea4_tests.log 2>&1 || { tail -30 $O/r14ea4_tests.log; exit 1; }
tail -1 $O/r14ea4_tests.log
bash tools/ab.sh --tag r14ea4 --rounds 2 -- "--workload evaluate_at --steps 3 --warmup 1" cur env:DPF_POINTS_ILP=2 || exit 1
bash tools/ab.sh --tag r14ea4s --rounds 2 -- "--workload evaluate_at_sum --steps 3 --warmup 1" cur env:DPF_POINTS_ILP=2 || exit 1
