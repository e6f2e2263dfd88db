set -u
L=distributed_point_functions_amd/lib/libdpf_hip.so
timeout -k 10 300 python tools/expand_ab.py --rounds 3 --reps 8 --variants vlib/head.so $L > gpurun_out/ab14.txt 2>&1; cat gpurun_out/ab14.txt
for r in 1 2; do
for v in 1 0; do
DPF_EXPAND_NO_OCTET=$v timeout -k 10 300 python bench.py --workload full_domain_tuple --tuple-type intmodn32x2 --steps 5 --warmup 1 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('no_octet=$v', d['ms_per_step'], d['roofline']['achieved'])"
done; done
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -m gpu -k "specialised or fast_types or generic or uneven" > gpurun_out/t_tup.log 2>&1; tail -2 gpurun_out/t_tup.log
