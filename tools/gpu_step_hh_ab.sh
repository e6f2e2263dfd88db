#!/bin/bash
# One lease: the tests touched by the batch-context / host-output changes, the
# heavy-hitters lean-kernel A/B at 2^18 clients, the drop-in API split probe,
# and a profile of the lean kernel.  Usage: bash tools/gpu_step_hh_ab.sh <tag>
set -u
TAG=${1:-r14a}
O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_batch_context_gpu.py tests/test_heavy_hitters_gpu.py \
  tests/test_api_gpu.py tests/test_cpp_api_gpu.py tests/test_host_copies_gpu.py -x -q \
  --timeout 240 --timeout-method thread > $O/${TAG}_tests.log 2>&1
rc=$?; tail -3 $O/${TAG}_tests.log; [ $rc -eq 0 ] || exit 1
for v in lean nolean lean2; do
  if [ $v = nolean ]; then export DPF_BATCH_NO_LEAN=1; else unset DPF_BATCH_NO_LEAN; fi
  timeout -k 10 200 python bench.py --workload heavy_hitters --keys-log 18 --no-cpu-baseline > $O/${TAG}_hh18_$v.json 2> $O/${TAG}_hh18_$v.err || { tail $O/${TAG}_hh18_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${TAG}_hh18_$v.json'));print('$v', d['seconds_per_pass'], d['roofline']['achieved'], d['roofline']['frac'])"
done
unset DPF_BATCH_NO_LEAN
F='^BM_EvaluateRegularDpf<(uint64_t>/(20|22|24)|uint128>/(20|22)|Tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>>/(18|20|22)|Tuple<uint64_t, uint64_t>>/(18|20|22)|XorWrapper<uint128>>/(20|22))$'
timeout -k 10 300 distributed_point_functions_amd/lib/dpf_benchmark --split "--benchmark_filter=$F" > $O/${TAG}_split.txt 2>&1 || { tail $O/${TAG}_split.txt; exit 1; }
timeout -k 10 300 distributed_point_functions_amd/lib/dpf_benchmark "--benchmark_filter=^BM_EvaluateRegularDpf" > $O/${TAG}_regular.txt 2>&1 || { tail $O/${TAG}_regular.txt; exit 1; }
cat $O/${TAG}_split.txt
bash tools/profile_workload.sh $TAG hh18 "hh_level_kernel" total:2 -- --workload heavy_hitters --keys-log 18 --no-cpu-baseline
