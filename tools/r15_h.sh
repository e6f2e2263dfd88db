#!/bin/bash
# r15 lease H: where small full-domain calls spend their time.
#   EvaluateUntil host phases (DPF_HOST_TIMING) for BM_EvaluateRegularDpf<uint64_t>/12, /16, /20;
#   kernel trace of config 1 (log 20) and of the /12 call.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
B=distributed_point_functions_amd/lib/dpf_benchmark
for l in 12 16 20; do
  DPF_HOST_TIMING=1 timeout -k 10 120 $B "--benchmark_filter=EvaluateRegularDpf<uint64_t>/$l\$" > $O/r15h_timing_$l.txt 2>&1 || exit 1
  grep -h "BM_\|host timing" $O/r15h_timing_$l.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r15h_prof_c1 -o c1 -- python3 bench.py --log-domain 20 --steps 200 --warmup 20 --no-cpu-baseline > $O/r15h_c1.log 2>&1 || exit 1
find $O/r15h_prof_c1 -name "*kernel_stats.csv" -exec cat {} \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r15h_prof_12 -o b12 -- $B "--benchmark_filter=EvaluateRegularDpf<uint64_t>/12\$" > $O/r15h_b12.log 2>&1 || exit 1
find $O/r15h_prof_12 -name "*kernel_stats.csv" -exec cat {} \;
