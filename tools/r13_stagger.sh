#!/bin/bash
# Heavy-hitters pass (2^18 clients) with the upper 8 waves of each workgroup
# started late (DPF_BATCH_STAGGER x 8128 clocks) vs none; plus a one-rank
# RCCL smoke (init + all_reduce on cuda:0).
set -u
mkdir -p gpurun_out
for r in 1 2; do
  bash tools/ab_lib.sh "--workload heavy_hitters --keys-log 18" cur stag4 stag8 stag14 || exit 1
done
MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 RANK=0 WORLD_SIZE=1 timeout -k 10 120 python -c "
import torch, torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group('nccl', device_id=torch.device('cuda', 0))
t = torch.ones(4, device='cuda'); dist.all_reduce(t); torch.cuda.synchronize()
print('rccl one-rank all_reduce ok', t.tolist(), dist.get_backend())
dist.destroy_process_group()
"
