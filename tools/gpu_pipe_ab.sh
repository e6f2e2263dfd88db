#!/bin/bash
# r14 A/B of the large host-output path: (1) the first call's expansion as 8
# subtree launches whose copies overlap the later launches (default) vs one
# launch (DPF_EVAL_SPLIT=0); (2) pipelined map+register of the fresh vector
# (default) vs the whole range first (DPF_HIP_D2H_PIPELINE=0).
set -u
bash tools/ab.sh --tag r14split --rounds 2 --tests "tests/test_api_gpu.py::test_pipelined_host_output_and_its_fallbacks tests/test_api_gpu.py::test_split_first_call_then_next_level tests/test_api_gpu.py::test_concurrent_pipelined_host_outputs tests/test_api_gpu.py::test_large_host_output_matches_device tests/test_api_gpu.py::test_concurrent_large_host_outputs tests/test_host_copies_gpu.py" -- "--host-output --steps 3 --warmup 1" cur env:DPF_EVAL_SPLIT=0 env:DPF_HIP_D2H_PIPELINE=0 || exit 1
bash tools/ab.sh --tag r14split128 --rounds 2 -- "--workload full_domain_u128 --host-output --steps 2 --warmup 1" cur env:DPF_EVAL_SPLIT=0 || exit 1
