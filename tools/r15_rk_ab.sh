#!/bin/bash
# r15 lease A2 (the GPU suite passed on this tree: profiles/r15a_gpu_tests.log):
# same-box A/B of the round-key form -- lane-resident VGPRs read by
# v_readlane (vlib/rk1.so, -DDPF_RK_LANES=1) vs the kernel-argument s_load
# form (cur) -- and of the vector-L1 second lookup engine (round 1 of every
# AES from a 1 KiB T0 table through the vector memory pipe, vlib/mi1.so, vs
# vlib/mi0.so: both built with the max-ilp scheduler, since iterative-ilp
# crashes hipcc's register allocator on the L1 variant); then the
# mapped-range registration threshold and the EvaluateAt host path.
set -u
O=gpurun_out; mkdir -p $O
bash tools/ab.sh --tag r15a_fd --rounds 2 -- "" cur lib:mi0 lib:mi1 || exit 1
bash tools/ab.sh --tag r15a_fdrk --rounds 2 -- "" cur lib:rk1 || echo "fd rk1 failed"
bash tools/ab.sh --tag r15a_tup --rounds 2 -- "--workload full_domain_tuple" cur lib:rk1 || echo "tup rk1 failed"
bash tools/ab.sh --tag r15a_dcf --rounds 2 -- "--workload dcf" cur lib:rk1 || echo "dcf rk1 failed"
bash tools/ab.sh --tag r15a_ea --rounds 2 -- "--workload evaluate_at --keys-log 18" cur lib:mi0 lib:mi1 || exit 1
timeout -k 10 300 python tools/mapped_copy_ab.py > $O/r15a_mapped_copy.jsonl 2>&1; echo "mapped rc=$?"
DPF_HOST_TIMING=1 timeout -k 10 300 distributed_point_functions_amd/lib/dpf_benchmark --benchmark_filter=BatchEvaluation \
  > $O/r15a_batch_evaluation.txt 2>&1; echo "batch_evaluation rc=$?"; cat $O/r15a_batch_evaluation.txt
