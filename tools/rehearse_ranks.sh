export DPF_BENCH_ONE_GPU=1
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 240 $R --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/n2_fd.log 2>&1 && \
timeout -k 10 240 $R --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --workload full_domain_u128 > gpurun_out/n2_u128.log 2>&1 && \
timeout -k 10 240 $R --master-port 29513 bench.py --gpus 2 --steps 2 --warmup 1 --workload evaluate_at_sum --keys-log 18 > gpurun_out/n2_eas.log 2>&1 && \
timeout -k 10 240 $R --master-port 29514 bench.py --gpus 2 --steps 2 --warmup 1 --workload evaluate_at --keys-log 18 > gpurun_out/n2_ea.log 2>&1 && \
timeout -k 10 300 $R --master-port 29515 bench.py --gpus 2 --workload heavy_hitters --keys-log 16 > gpurun_out/n2_hh.log 2>&1 && \
timeout -k 10 240 $R --master-port 29516 bench.py --gpus 2 --steps 2 --warmup 1 --workload dcf --dcf-keys-log 14 > gpurun_out/n2_dcf.log 2>&1
