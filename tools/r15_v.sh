#!/bin/bash
# r15 lease V (diagnostic): where BM_EvaluateHierarchicalFull's calls spend
# their time (DPF_HOST_TIMING EvaluateUntil phases), plus a kernel trace.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
B=distributed_point_functions_amd/lib/dpf_benchmark
for t in uint8_t uint64_t; do
  DPF_HOST_TIMING=1 timeout -k 10 120 $B "--benchmark_filter=HierarchicalFull<$t>/15\$" > $O/r15v_hf_$t.txt 2>&1 || exit 1
  grep -h "BM_\|host timing" $O/r15v_hf_$t.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r15v_prof -o hf -- $B '--benchmark_filter=HierarchicalFull<uint64_t>/15$' > $O/r15v_prof.log 2>&1 || exit 1
find $O/r15v_prof -name "*kernel_stats.csv" -exec cut -c1-150 {} \;
