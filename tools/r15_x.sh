#!/bin/bash
# r15 lease X: EvaluateUntil prefix dedup into vectors kept across calls, identity
# check and gather offsets on host threads (on top of lease W: one-image walk)
# control bits, paths and correction words; read in place when small) and one
# D2H back for the context, parallel prefix range check -- parity, then the
# hierarchical rows of the reference grid with the host-phase split.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
B=distributed_point_functions_amd/lib/dpf_benchmark
timeout -k 10 900 python -u -m pytest tests/test_api_gpu.py tests/test_cpp_api_gpu.py tests/test_reference_benchmarks_gpu.py \
  tests/test_key_batch_gpu.py tests/test_dcf_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r15x_tests.log 2>&1
rc=$?; tail -2 $O/r15x_tests.log; [ $rc -eq 0 ] || { tail -30 $O/r15x_tests.log; exit 1; }
for t in uint8_t uint64_t; do
  DPF_HOST_TIMING=1 timeout -k 10 120 $B "--benchmark_filter=HierarchicalFull<$t>/15\$" > $O/r15x_hf_$t.txt 2>&1 || exit 1
  grep -h "BM_\|host timing" $O/r15x_hf_$t.txt
done
timeout -k 10 300 $B '--benchmark_filter=HierarchicalFull|IsrgExample|HeavyHitters' > $O/r15x_grid.txt 2>&1 || exit 1
grep BM_ $O/r15x_grid.txt
timeout -k 10 300 python bench.py --workload synthetic_hierarchical --domain 32 > $O/r15x_syn_h32.json 2> $O/r15x_syn_h32.err || exit 1
python3 -c "import json; d=json.loads(open('$O/r15x_syn_h32.json').read().strip().splitlines()[-1]); print('syn_h32', d['value'], d['unit'])"
