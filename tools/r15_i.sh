#!/bin/bash
# r15 lease I: latency-mode full-domain expansion of small trees
# (expand_small_kernel) -- parity, config 1 with it on/off, the small end of
# the reference grid on/off, and config 1's kernel trace.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_api_gpu.py tests/test_cpp_api_gpu.py \
  tests/test_reference_benchmarks_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r15i_tests.log 2>&1
rc=$?; tail -2 $O/r15i_tests.log; [ $rc -eq 0 ] || { tail -30 $O/r15i_tests.log; exit 1; }
for r in 1 2; do
  for v in 1 0; do
    DPF_EXPAND_SMALL=$v timeout -k 10 200 python bench.py --log-domain 20 --steps 500 --warmup 50 --no-cpu-baseline \
      > $O/r15i_c1_s${v}_r$r.json 2> $O/r15i_c1_s${v}_r$r.err || { tail $O/r15i_c1_s${v}_r$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step']*1e3, 'us/step', d['roofline']['launch_ms']*1e3, 'us launch')" $O/r15i_c1_s${v}_r$r.json small=$v
  done
done
B=distributed_point_functions_amd/lib/dpf_benchmark
for v in 1 0; do
  DPF_EXPAND_SMALL=$v timeout -k 10 300 $B '--benchmark_filter=EvaluateRegularDpf<(uint8_t|uint64_t|uint128|XorWrapper<uint128>)>/(12|14|16|18|20)$' \
    > $O/r15i_grid_s$v.txt 2>&1 || exit 1
  echo "small=$v"; grep BM_ $O/r15i_grid_s$v.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r15i_prof_c1 -o c1 -- python3 bench.py --log-domain 20 --steps 200 --warmup 20 --no-cpu-baseline > $O/r15i_prof_c1.log 2>&1 || exit 1
find $O/r15i_prof_c1 -name "*kernel_stats.csv" -exec cat {} \;
