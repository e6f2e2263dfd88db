#!/bin/bash
# r15 lease A: the GPU suite on the in-tree build, then round keys as
# lane-resident VGPRs (v_readlane, DPF_RK_LANES=1: vlib/rk1.so) vs the
# kernel-argument s_load form (vlib/rk0.so, -DDPF_RK_LANES=0), same box, every
# AES kernel class; then the mapped-host-range registration threshold A/B.
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/r15a_tests.log 2>&1
rc=$?; tail -3 $O/r15a_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab.sh --tag r15a_fd --rounds 2 -- "" lib:rk1 lib:rk0 || exit 1
bash tools/ab.sh --tag r15a_tup --rounds 2 -- "--workload full_domain_tuple" lib:rk1 lib:rk0 || exit 1
bash tools/ab.sh --tag r15a_dcf --rounds 2 -- "--workload dcf" lib:rk1 lib:rk0 || exit 1
bash tools/ab.sh --tag r15a_ea --rounds 2 -- "--workload evaluate_at --keys-log 18" lib:rk1 lib:rk0 || exit 1
timeout -k 10 300 python tools/mapped_copy_ab.py > $O/r15a_mapped_copy.jsonl 2>&1; echo "mapped rc=$?"
# EvaluateAt host path: per-phase timing and the reference grid's BatchEvaluation
DPF_HOST_TIMING=1 timeout -k 10 300 distributed_point_functions_amd/lib/dpf_benchmark --benchmark_filter=BatchEvaluation \
  > $O/r15a_batch_evaluation.txt 2>&1; echo "batch_evaluation rc=$?"; cat $O/r15a_batch_evaluation.txt
