set -u
L=distributed_point_functions_amd/lib/libdpf_hip.so
B=distributed_point_functions_amd/lib/dpf_benchmark
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r09b_gpu_tests.log 2>&1 || exit 1
for v in old new old new; do
  cp vlib/$v.so $L
  timeout -k 10 120 $B '--benchmark_filter=BatchEvaluation|EvaluateRegularDpf<uint64_t>/12' > gpurun_out/ab_batch_$v.txt 2>&1 || exit 1
  cat gpurun_out/ab_batch_$v.txt >> gpurun_out/ab_batch_all.txt
done
cp vlib/new.so $L
