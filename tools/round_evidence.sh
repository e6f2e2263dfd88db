#!/bin/bash
# One GPU lease's worth of round evidence, so every committed number comes
# from the same box and tree:
#   1. the -m gpu suite and smoke();
#   2. the default bench line (no profiler);
#   3. the API-level lines (--host-output) for configs 2 and 3 (one shard);
#   4. the rocprofv3 kernel trace + PMC passes of the SAME bench command
#      (20 timed steps after 3 warmups; tools/pmc_summary.py --skip 3 averages
#      exactly the timed launches);
#   5. the reference's benchmark suite restated on the drop-in API.
# Usage (GPU box, repo root): bash tools/round_evidence.sh <tag> [--no-tests]
set -u
TAG=${1:-r12}
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
if [ "${2:-}" != "--no-tests" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/${TAG}_gpu_tests.log; exit 1; }
  tail -2 $O/${TAG}_gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/${TAG}_smoke.log 2>&1 || { cat $O/${TAG}_smoke.log; exit 1; }
  cat $O/${TAG}_smoke.log
fi
timeout -k 10 300 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { tail -20 $O/${TAG}_bench.err; exit 1; }
cat $O/${TAG}_bench.json
timeout -k 10 300 python bench.py --host-output --no-cpu-baseline --steps 5 --warmup 1 > $O/${TAG}_api_u64.json 2> $O/${TAG}_api_u64.err || { tail -20 $O/${TAG}_api_u64.err; exit 1; }
timeout -k 10 400 python bench.py --workload full_domain_u128 --host-output --no-cpu-baseline --steps 3 --warmup 1 > $O/${TAG}_api_u128.json 2> $O/${TAG}_api_u128.err || { tail -20 $O/${TAG}_api_u128.err; exit 1; }
echo "api lines ok"
bash profiles/profile.sh $TAG --steps 20 --warmup 3 --no-cpu-baseline || exit 1
timeout -k 10 600 distributed_point_functions_amd/lib/dpf_benchmark > $O/${TAG}_reference_benchmarks.txt 2> $O/${TAG}_reference_benchmarks.err || { tail -5 $O/${TAG}_reference_benchmarks.err; exit 1; }
echo "all ok"
