export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_batch_context_gpu.py tests/test_heavy_hitters_gpu.py tests/test_key_batch_gpu.py tests/test_kernels_gpu.py tests/test_api_gpu.py tests/test_cpp_api_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r16h_tests.log 2>&1; rc=$?; tail -2 $O/r16h_tests.log; [ $rc -eq 0 ] || exit 1
for d in 128 32; do
  DPF_BATCH_HOST_TIMING=1 timeout -k 10 300 python bench.py --workload synthetic_hierarchical_device --domain $d > $O/r16h_syn_dev$d.json 2> $O/r16h_syn_dev$d.err || exit 1
  DPF_HOST_TIMING=1 timeout -k 10 300 python bench.py --workload synthetic_hierarchical --domain $d > $O/r16h_syn_h$d.json 2> $O/r16h_syn_h$d.err || exit 1
done
bash tools/ab.sh --tag r16h_fd --rounds 2 -- "--no-host-output --steps 20" cur env:DPF_EXPAND_TOP=0 || exit 1
bash tools/ab.sh --tag r16h_r8 --rounds 2 -- "--rehearse-world 8 --no-host-output --steps 50" cur env:DPF_EXPAND_TOP=0 || exit 1
bash tools/ab.sh --tag r16h_hh20 --rounds 1 -- "--workload heavy_hitters" cur lib:hhnt || exit 1
