#!/bin/bash
# r13 A/B on one lease: DCF fast kernel (one / two items per lane) and the
# batch kernel's key-pair prefetch / iterative-ilp build against HEAD's
# library (vlib/base.so), after the parity tests of the changed kernels.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_dcf_gpu.py tests/test_batch_context_gpu.py tests/test_heavy_hitters_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r13_tests.log 2>&1 || { tail -30 $O/r13_tests.log; exit 1; }
tail -2 $O/r13_tests.log
for r in 1 2; do
  bash tools/ab_lib.sh "--workload dcf --steps 10 --warmup 2" base cur d2 || exit 1
done
DPF_DCF_GENERAL=1 timeout -k 10 300 python bench.py --workload dcf --steps 10 --warmup 2 --no-cpu-baseline > $O/r13_dcf_general.json 2>&1 || exit 1
python -c "import json; d=json.loads([l for l in open('$O/r13_dcf_general.json') if l.startswith('{')][0]); print('general-on-cur', d['value'], d['roofline']['launch_ms'])"
for r in 1 2; do
  bash tools/ab_lib.sh "--workload heavy_hitters --keys-log 18" base cur nopf bilp || exit 1
done
echo all ok
