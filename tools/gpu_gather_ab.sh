#!/bin/bash
# r14 A/B: heavy hitters' start-seed gather with four keys' loads in flight
# per lane (default) vs one (DPF_BATCH_GATHER_KEYS=1).  Parity first: the
# batch-context tests (in-place gather path included) and heavy hitters.
set -u
bash tools/ab.sh --tag r14gather --rounds 2 --tests "tests/test_batch_context_gpu.py tests/test_heavy_hitters_gpu.py" -- "--workload heavy_hitters" cur env:DPF_BATCH_GATHER_KEYS=1 || exit 1
