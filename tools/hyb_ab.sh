#!/bin/bash
# Expand-kernel A/B on one box: parity tests of the hybrid shapes, then
# tools/variant_bench.py per library.  Args: name[:ENV=VAL] (vlib/name.so with
# that environment, e.g. hyb_w2:DPF_EXPAND_HYBRID=1 for the hybrid path).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "hybrid or fast_types" -x -q --timeout 120 --timeout-method thread > gpurun_out/hyb_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/hyb_tests.log; exit 1; }
tail -2 gpurun_out/hyb_tests.log
for a in "$@"; do
  l=${a%%:*}; e=""; [ "$a" != "$l" ] && e=${a#*:}
  echo -n "$a "
  env $e timeout -k 10 200 python tools/variant_bench.py --lib vlib/$l.so | sed 's/^[^ ]* //' || exit 1
done
