#!/bin/bash
# r15 lease S: where small point launches should switch from lane chains to
# lane quads -- BM_BatchEvaluation at DPF_POINTS_QUAD_MAX = default (num_cus x 64
# = 16384 points), 65536, 524288; two rounds; plus the points quad parity tests
# with the cut-over raised.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
B=distributed_point_functions_amd/lib/dpf_benchmark
DPF_POINTS_QUAD_MAX=524288 timeout -k 10 600 python -u -m pytest tests/test_key_batch_gpu.py tests/test_api_gpu.py -x -q \
  -k "quad or latency or evaluate_at" --timeout 300 --timeout-method thread > $O/r15s_tests.log 2>&1
rc=$?; tail -2 $O/r15s_tests.log; [ $rc -eq 0 ] || { tail -30 $O/r15s_tests.log; exit 1; }
for r in 1 2; do
  for m in 0 65536 524288; do
    if [ $m = 0 ]; then unset DPF_POINTS_QUAD_MAX; else export DPF_POINTS_QUAD_MAX=$m; fi
    timeout -k 10 200 $B '--benchmark_filter=BM_BatchEvaluation' > $O/r15s_be_${m}_r$r.txt 2>&1 || exit 1
    grep BM_ $O/r15s_be_${m}_r$r.txt | sed -E 's/ +([0-9]+) ns.*/ \1/' | awk -v m=$m '{print "max=" m, $0}'
  done
done
