#!/bin/bash
# Point-kernel quad (ILP4) check: the point tests with the quad kernel, then
# bench.py --workload evaluate_at with pairs (DPF_POINTS_QUAD=0) and quads.
set -u
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py -k "points" tests/test_key_batch_gpu.py tests/test_fullsize_gpu.py -k "points or config4 or evaluate_at" \
  > gpurun_out/quad_tests.log 2>&1 || { tail -30 gpurun_out/quad_tests.log; exit 1; }
tail -3 gpurun_out/quad_tests.log
for v in 0 1 0 1; do
  DPF_POINTS_QUAD=$v timeout -k 10 300 python bench.py --workload evaluate_at --no-cpu-baseline \
    > gpurun_out/quad_$v.log 2>&1 || exit 1
  python -c "import json; d=json.loads([l for l in open('gpurun_out/quad_$v.log') if l.startswith('{')][0]); print('quad=$v', d['value'], d['unit'], d.get('roofline',{}).get('launch_ms'))"
done
