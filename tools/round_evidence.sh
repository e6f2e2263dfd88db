#!/bin/bash
# A round's evidence, on the final tree, in four leases (each under gpurun's
# 20-minute limit).  Every number in DESIGN.md / README.md cites these files.
# Each bench line is taken in the SAME lease as its workload's profile, right
# after it (the profile is copied into profiles/ on the box first, so the line's
# `roofline.profiled_launch_ms` / `profile_vs_launch` compare one box with
# itself; boxes differ by several percent in sustained clock).
#   part1: the -m gpu suite, smoke(), config 2's profile and its default bench
#          line (with the CPU baselines), the API-level lines (--host-output)
#          for configs 2 and 3, and the reference's benchmark suite on the
#          drop-in API (default allocator and --malloc_keep_pages);
#   part2: profile + bench line of config 3 (uint128) and the two tuple kernels;
#   part3: profile + bench line of config 4 (EvaluateAt per key and summed) and DCF;
#   part4: profile + bench line of config 5b (heavy hitters), then config 1's
#          line (log 20, latency mode) and the synthetic-benchmark lines (no
#          kernel profile of their own).
# Each profile is tools/profile_workload.sh: a kernel trace and four PMC
# passes of the SAME bench command, summarised per workload into
# gpurun_out/<tag>_<workload>_summary.json (copied to profiles/ afterwards).
# Usage (GPU box, repo root): bash tools/round_evidence.sh <tag> part1|part2|part3|part4
set -u
TAG=${1:-r16}; PART=${2:-part1}
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
prof() { bash tools/profile_workload.sh "$@" || exit 1; }
# bench line <name> <bench.py args...> -> $O/bench_<tag>_<name>.json
line() {
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > $O/bench_${TAG}_$name.log 2>&1 || { tail $O/bench_${TAG}_$name.log; exit 1; }
  grep '^{' $O/bench_${TAG}_$name.log > $O/bench_${TAG}_$name.json
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); r=d.get('roofline',{}); print(sys.argv[2], d['value'], d['unit'], 'frac', r.get('frac'), 'profile_vs_launch', r.get('profile_vs_launch'))" $O/bench_${TAG}_$name.json $name
}
# profile a workload, make its summary the one bench.py quotes, then its bench line:
#   profline <workload tag> '<kernel>' <mode> <line name> '<profile-only args>' <bench.py args...>
profline() {
  local wl=$1 kern=$2 mode=$3 name=$4 pargs=$5; shift 5
  prof $TAG $wl "$kern" $mode -- "$@" $pargs
  cp $O/${TAG}_${wl}_summary.json profiles/ || exit 1
  line $name "$@"
}
case $PART in
part1)
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/${TAG}_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/${TAG}_gpu_tests.log; exit 1; }
  tail -2 $O/${TAG}_gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/${TAG}_smoke.log 2>&1 || { cat $O/${TAG}_smoke.log; exit 1; }
  cat $O/${TAG}_smoke.log
  prof $TAG full_domain "expand_octet_kernel<FastIntLeaf<64, false> >" launch:3 -- --steps 20 --warmup 3 --no-cpu-baseline --no-host-output
  cp $O/${TAG}_full_domain_summary.json profiles/ || exit 1
  timeout -k 10 300 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { tail -20 $O/${TAG}_bench.err; exit 1; }
  cat $O/${TAG}_bench.json
  timeout -k 10 300 python bench.py --host-output --no-cpu-baseline --steps 5 --warmup 1 > $O/${TAG}_api_u64.json 2> $O/${TAG}_api_u64.err || { tail -20 $O/${TAG}_api_u64.err; exit 1; }
  timeout -k 10 500 python bench.py --workload full_domain_u128 --host-output --host-output-reps 6 --no-cpu-baseline --steps 3 --warmup 1 > $O/${TAG}_api_u128.json 2> $O/${TAG}_api_u128.err || { tail -20 $O/${TAG}_api_u128.err; exit 1; }
  echo "api lines ok"
  # The shard each rank of a 2/4/8-GPU run evaluates (strong scaling), on this GPU.
  for w in 2 4 8; do
    timeout -k 10 200 python bench.py --rehearse-world $w --no-cpu-baseline --no-host-output --steps 50 > $O/${TAG}_rehearse$w.json 2>> $O/${TAG}_bench.err || exit 1
  done
  timeout -k 10 600 distributed_point_functions_amd/lib/dpf_benchmark > $O/${TAG}_reference_benchmarks.txt 2> $O/${TAG}_reference_benchmarks.err || { tail -5 $O/${TAG}_reference_benchmarks.err; exit 1; }
  timeout -k 10 300 distributed_point_functions_amd/lib/dpf_benchmark --malloc_keep_pages "--benchmark_filter=^BM_EvaluateRegularDpf" > $O/${TAG}_reference_benchmarks_keep_pages.txt 2>&1 || exit 1
  ;;
part2)
  profline full_domain_u128 "expand_octet_kernel<FastIntLeaf<128, false> >" launch:2 full_domain_u128 "--steps 10 --warmup 2 --no-cpu-baseline --no-host-output" --workload full_domain_u128
  profline full_domain_tuple_intmodn32x2 "expand_octet_kernel<Mod32Leaf<2> >" launch:2 tuple_mod "--steps 10 --warmup 2 --no-cpu-baseline" --workload full_domain_tuple --tuple-type intmodn32x2
  profline full_domain_tuple_u32x2 "expand_octet_kernel<FastIntLeaf<32, false> >" launch:2 tuple_u32 "--steps 10 --warmup 2 --no-cpu-baseline" --workload full_domain_tuple --tuple-type u32x2
  ;;
part3)
  profline evaluate_at "eval_points4_kernel" launch:1 evaluate_at "--steps 3 --warmup 1 --no-cpu-baseline" --workload evaluate_at
  profline evaluate_at_sum "eval_points4_kernel" launch:1 evaluate_at_sum "--steps 3 --warmup 1 --no-cpu-baseline" --workload evaluate_at_sum
  profline dcf "dcf_fast_kernel" launch:2 dcf "--steps 10 --warmup 2 --no-cpu-baseline" --workload dcf
  ;;
part4)
  PROFILE_PASS_LIMIT=400 profline heavy_hitters "hh_keys_kernel|hh_key_table_kernel|batch_level_kernel<Mod32V<2, true>, 2, true>|gather_seeds_im_kernel|finalize_sums_kernel" total:2 heavy_hitters "--no-cpu-baseline" --workload heavy_hitters
  line config1 --log-domain 20 --steps 2000 --warmup 5000   # ~0.3 s of warmup: the GPU at full clock
  line syn_dev32 --workload synthetic_hierarchical_device --domain 32
  line syn_dev128 --workload synthetic_hierarchical_device --domain 128
  line syn_h32 --workload synthetic_hierarchical --domain 32
  line syn_h128 --workload synthetic_hierarchical --domain 128
  line syn_d32 --workload synthetic_direct --domain 32
  line syn_d128 --workload synthetic_direct --domain 128
  ;;
esac
echo "$PART ok"
