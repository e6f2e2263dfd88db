#!/bin/bash
# r15 lease C: GPU suite on the host worker pool build, then the EvaluateAt
# host-path phases per reference-benchmark case and the whole reference grid.
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/r15c_tests.log 2>&1
rc=$?; tail -3 $O/r15c_tests.log; [ $rc -eq 0 ] || exit 1
for c in 1/400000 10/40000 100/4000; do
  DPF_HOST_TIMING=1 timeout -k 10 120 distributed_point_functions_amd/lib/dpf_benchmark \
    --benchmark_filter="BatchEvaluation.*/$c\$" > $O/r15c_be_${c/\//_}.txt 2>&1 || exit 1
  cat $O/r15c_be_${c/\//_}.txt
done
timeout -k 10 600 distributed_point_functions_amd/lib/dpf_benchmark > $O/r15c_reference_benchmarks.txt 2>&1
echo "grid rc=$?"; tail -5 $O/r15c_reference_benchmarks.txt
