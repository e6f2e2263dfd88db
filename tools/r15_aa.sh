#!/bin/bash
# r15 lease AA (diagnostic): EvaluateUntil's host phases with the validation
# and the prefix dedup split, HierarchicalFull/15 and synthetic hierarchical.
set -u
O=gpurun_out; mkdir -p $O
B=distributed_point_functions_amd/lib/dpf_benchmark
for t in uint8_t uint64_t; do
  DPF_HOST_TIMING=1 timeout -k 10 120 $B "--benchmark_filter=HierarchicalFull<$t>/15\$" > $O/r15aa_hf_$t.txt 2>&1 || exit 1
  grep -h "BM_\|host timing" $O/r15aa_hf_$t.txt
done
DPF_HOST_TIMING=1 DPF_BATCH_HOST_TIMING=1 timeout -k 10 300 python bench.py --workload synthetic_hierarchical --domain 32 > $O/r15aa_syn.json 2> $O/r15aa_syn.err || exit 1
grep -h "host timing" $O/r15aa_syn.err
