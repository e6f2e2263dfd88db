#!/bin/bash
# A round's evidence, on the final tree, in four leases (each under gpurun's
# 20-minute limit).  Every number in DESIGN.md / README.md cites these files.
#   part1: the -m gpu suite, smoke(), the default bench line (config 2, with
#          its CPU baselines), the API-level lines (--host-output) for configs
#          2 and 3, and the reference's benchmark suite on the drop-in API;
#   part2: every bench.py workload once (tools/bench_all.sh, CPU baselines
#          included);
#   part3: the rocprof evidence of configs 2 and 3 and the two tuple kernels;
#   part4: the rocprof evidence of configs 4 (per key, summed), 5b and DCF.
# Each profile is tools/profile_workload.sh: a kernel trace and four PMC
# passes of the SAME bench command, summarised per workload into
# gpurun_out/<tag>_<workload>_summary.json (copied to profiles/ afterwards).
# Usage (GPU box, repo root): bash tools/round_evidence.sh <tag> part1|part2|part3|part4
set -u
TAG=${1:-r14}; PART=${2:-part1}
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
prof() { bash tools/profile_workload.sh "$@" || exit 1; }
case $PART in
part1)
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/${TAG}_gpu_tests.log; exit 1; }
  tail -2 $O/${TAG}_gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/${TAG}_smoke.log 2>&1 || { cat $O/${TAG}_smoke.log; exit 1; }
  cat $O/${TAG}_smoke.log
  timeout -k 10 300 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { tail -20 $O/${TAG}_bench.err; exit 1; }
  cat $O/${TAG}_bench.json
  timeout -k 10 300 python bench.py --host-output --no-cpu-baseline --steps 5 --warmup 1 > $O/${TAG}_api_u64.json 2> $O/${TAG}_api_u64.err || { tail -20 $O/${TAG}_api_u64.err; exit 1; }
  timeout -k 10 400 python bench.py --workload full_domain_u128 --host-output --no-cpu-baseline --steps 3 --warmup 1 > $O/${TAG}_api_u128.json 2> $O/${TAG}_api_u128.err || { tail -20 $O/${TAG}_api_u128.err; exit 1; }
  echo "api lines ok"
  timeout -k 10 600 distributed_point_functions_amd/lib/dpf_benchmark > $O/${TAG}_reference_benchmarks.txt 2> $O/${TAG}_reference_benchmarks.err || { tail -5 $O/${TAG}_reference_benchmarks.err; exit 1; }
  timeout -k 10 300 distributed_point_functions_amd/lib/dpf_benchmark --malloc_keep_pages "--benchmark_filter=^BM_EvaluateRegularDpf" > $O/${TAG}_reference_benchmarks_keep_pages.txt 2>&1 || exit 1
  ;;
part2)
  [ -s $O/${TAG}_reference_benchmarks_keep_pages.txt ] || timeout -k 10 300 distributed_point_functions_amd/lib/dpf_benchmark --malloc_keep_pages "--benchmark_filter=^BM_EvaluateRegularDpf" > $O/${TAG}_reference_benchmarks_keep_pages.txt 2>&1 || exit 1
  bash tools/bench_all.sh $TAG || exit 1
  ;;
part3)
  prof $TAG full_domain "expand_octet_kernel<FastIntLeaf<64, false> >" launch:3 -- --steps 20 --warmup 3 --no-cpu-baseline
  prof $TAG full_domain_u128 "expand_octet_kernel<FastIntLeaf<128, false> >" launch:2 -- --workload full_domain_u128 --steps 10 --warmup 2 --no-cpu-baseline
  prof $TAG full_domain_tuple_intmodn32x2 "expand_octet_kernel<Mod32Leaf<2> >" launch:2 -- --workload full_domain_tuple --tuple-type intmodn32x2 --steps 10 --warmup 2 --no-cpu-baseline
  prof $TAG full_domain_tuple_u32x2 "expand_octet_kernel<FastIntLeaf<32, false> >" launch:2 -- --workload full_domain_tuple --tuple-type u32x2 --steps 10 --warmup 2 --no-cpu-baseline
  ;;
part4)
  timeout -k 10 400 python bench.py --workload heavy_hitters > $O/bench_${TAG}_heavy_hitters.log 2>&1 || { tail $O/bench_${TAG}_heavy_hitters.log; exit 1; }
  grep '^{' $O/bench_${TAG}_heavy_hitters.log > $O/bench_${TAG}_heavy_hitters.json
  prof $TAG evaluate_at "eval_points_kernel" launch:1 -- --workload evaluate_at --steps 3 --warmup 1 --no-cpu-baseline
  prof $TAG evaluate_at_sum "eval_points_kernel" launch:1 -- --workload evaluate_at_sum --steps 3 --warmup 1 --no-cpu-baseline
  prof $TAG dcf "dcf_fast_kernel" launch:2 -- --workload dcf --steps 10 --warmup 2 --no-cpu-baseline
  PROFILE_PASS_LIMIT=400 prof $TAG heavy_hitters "hh_level_kernel|batch_level_kernel<Mod32V<2, true>, 2, true>|gather_seeds_kernel|finalize_sums_kernel" total:2 -- --workload heavy_hitters --no-cpu-baseline
  ;;
esac
echo "$PART ok"
