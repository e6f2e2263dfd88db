#!/bin/bash
# r15 lease R: the small-call copy-mode parity tests, then evidence part 4 on
# the final tree (heavy hitters with the slot-table load hoisted).
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_api_gpu.py tests/test_dcf_gpu.py -x -q -k "copy_modes or large_domain" \
  --timeout 300 --timeout-method thread > $O/r15r_tests.log 2>&1
rc=$?; tail -2 $O/r15r_tests.log; [ $rc -eq 0 ] || { tail -30 $O/r15r_tests.log; exit 1; }
bash tools/round_evidence.sh r15 part4
