#!/bin/bash
# Short lease: batch-context + heavy-hitters GPU tests, the heavy-hitters
# lean/general A/B at 2^18 clients, and the fresh-output microbenchmark.
# Usage: bash tools/gpu_step_quick.sh <tag>
set -u
TAG=${1:-r14b}
O=gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_batch_context_gpu.py tests/test_heavy_hitters_gpu.py -x -q \
  --timeout 240 --timeout-method thread > $O/${TAG}_tests.log 2>&1
rc=$?; tail -2 $O/${TAG}_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab.sh --tag ${TAG}_hh18 --rounds 2 -- "--workload heavy_hitters --keys-log 18" cur env:DPF_BATCH_NO_LEAN=1 || exit 1
timeout -k 10 300 tools/fresh_output_microbench > $O/${TAG}_fresh_output.jsonl 2>&1 || exit 1
grep -E '"mib": (32|64)' $O/${TAG}_fresh_output.jsonl
timeout -k 10 120 tools/wsfbs_microbench > $O/${TAG}_wsfbs.jsonl 2>&1; echo "wsfbs rc=$?"; cat $O/${TAG}_wsfbs.jsonl
