#!/bin/bash
# One GPU call's worth of round evidence: the -m gpu suite, smoke(), the
# default bench line, then the rocprofv3 passes of profiles/profile.sh.
# Usage: bash tools/gpu_round_check.sh <tag>
TAG=${1:-r11}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { echo "gpu tests rc=$?" >> gpurun_out/${TAG}_gpu_tests.log; tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
cat gpurun_out/${TAG}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cat gpurun_out/${TAG}_bench.json
bash profiles/profile.sh $TAG || exit 1
