#!/bin/bash
# One GPU call's worth of round evidence: the -m gpu suite, then bench lines.
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests2.log 2>&1 || { echo "gpu tests rc=$?" >> gpurun_out/gpu_tests2.log; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_fd.log 2>&1 || exit 1
bash profiles/profile.sh r10b || exit 1
