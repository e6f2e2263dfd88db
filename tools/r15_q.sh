#!/bin/bash
# r15 lease Q: hh_level_kernel with its divisors and per-key pointers pinned in SGPRs
# (DPF_HH_PIN_DIV=1, in-tree: no s_load reloads in the key loop) vs not
# (vlib/pin0.so): parity, then heavy hitters 2^20 (slot-table in place:
# scattered start seeds) and 2^18 (spare), same box.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_batch_context_gpu.py tests/test_heavy_hitters_gpu.py -x -q \
  --timeout 300 --timeout-method thread > $O/r15q_tests.log 2>&1
rc=$?; tail -2 $O/r15q_tests.log; [ $rc -eq 0 ] || { tail -30 $O/r15q_tests.log; exit 1; }
bash tools/ab.sh --tag r15q_hh20 --rounds 1 -- "--workload heavy_hitters --no-cpu-baseline" cur lib:pin0 || exit 1
bash tools/ab.sh --tag r15q_hh18 --rounds 2 -- "--workload heavy_hitters --keys-log 18 --no-cpu-baseline" cur lib:pin0 || exit 1
