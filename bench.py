#!/usr/bin/env python3
"""Headline benchmark: full-domain DPF evaluation, 2^30 uint64 leaves per GPU.

Metric (BASELINE.json): "DPF leaf evals/sec, full-domain 2^30 uint64 at
1/2/4/8 GPUs; AES blocks/s".  One *step* = one full-domain EvaluateUntil-
equivalent pass of one key over a 2^30-element uint64 domain per GPU: the
fused dpf_hip_expand kernel (ExpandSeeds + HashExpandedSeeds + correction,
SURVEY.md section 8a rows a4-a6, a12-a13) writing 8 GiB of corrected outputs
to HBM.  Inputs (key) are resident on the device before the timed region;
outputs stay device-resident (the PCIe-inclusive API rate is reported in
DESIGN.md, never as `value`).

Multi-GPU: weak scaling by subtree prefix.  With N ranks the
domain is 2^(30 + log2 N); rank g path-walks prefix g through the top log2 N
levels (dpf_hip_eval_paths, inside the timed step) and expands its own 2^30-leaf
subtree.  No collective on the data path; the timing max over ranks uses one
all_reduce outside the timed region.

Run: python bench.py [--gpus N --steps K --warmup W]
     torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

LOG_PER_GPU = 30          # 2^30 uint64 leaves per GPU (BASELINE.json configs[1])
AES_PEAK_GBLOCKS = 122.9  # integer-VALU AES roofline, SURVEY.md 8(d)
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-domain", type=int, default=LOG_PER_GPU)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-log", type=int, default=24,
                    help="log2 leaves of the bounded CPU oracle sample")
    return ap.parse_args()


def synthetic_key(rng, levels):
    """Synthetic key material: random root seed and correction words.  The
    evaluation work is independent of the key's values."""
    seed = rng.integers(0, 2**64, size=(1, 2), dtype=np.uint64)
    cws = rng.integers(0, 2**64, size=(levels, 2), dtype=np.uint64)
    cl = rng.integers(0, 2, size=levels, dtype=np.uint8)
    cr = rng.integers(0, 2, size=levels, dtype=np.uint8)
    vcw = rng.integers(0, 2**64, size=(2, 2), dtype=np.uint64)
    vcw[:, 1] = 0
    return seed, cws, cl, cr, vcw


def cpu_baseline(sample_log: int, levels_total: int):
    """Reference-faithful CPU restatement (oracle, OpenSSL EVP AES-NI, 64-block
    batches as dpf/distributed_point_function.cc:271-349), single thread, on a
    bounded subtree of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    rng = np.random.default_rng(1)
    D = sample_log - 1  # uint64: 2 elements per block
    seed, cws, cl, cr, vcw = synthetic_key(rng, D)
    ctrl = np.zeros(1, np.uint8)
    t0 = time.perf_counter()
    es, ec = O.expand_seeds(seed, ctrl, cws, cl, cr)
    out = O.hash_correct(("int", 64), es, ec, 1, 2, [[int(vcw[0, 0])], [int(vcw[1, 0])]], 0)
    dt = time.perf_counter() - t0
    leaves = out.shape[0]
    return {"value": leaves / dt, "unit": "leaves/s", "cores": 1, "kind": "port",
            "sample": f"2^{sample_log} uint64 leaves (one 2^{D}-block subtree, full ExpandSeeds+"
                      f"HashExpandedSeeds+correction), {dt:.2f} s on 1 host thread",
            "aes_blocks_per_s": (2 * (2**D - 1) + 2**D) / dt}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from distributed_point_functions_amd import hip_abi as H

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    H.load(require_gpu=True)
    dev = torch.device("cuda", local)
    stream = torch.cuda.current_stream(dev)

    k = int(round(math.log2(world))) if world > 1 else 0
    assert (1 << k) == world, "--gpus must be a power of two"
    log_domain = args.log_domain + k
    D_total = log_domain - 1            # uint64: tree depth = log_domain - 1 (proto_validator.cc:131-133)
    D = D_total - k                     # per-rank subtree depth
    rng = np.random.default_rng(1234)
    seed, cws, cl, cr, vcw = synthetic_key(rng, D_total)
    d_seed = H.to_device_blocks(seed, dev)
    d_ctrl = torch.zeros(1, dtype=torch.uint8, device=dev)
    d_cws = H.to_device_blocks(cws, dev)
    d_cl = H.to_device_u8(cl, dev)
    d_cr = H.to_device_u8(cr, dev)
    d_vcw = H.to_device_blocks(vcw, dev)
    d_path = H.to_device_blocks(np.array([[rank, 0]], np.uint64), dev)
    sub_seed = torch.empty_like(d_seed)
    sub_ctrl = torch.empty_like(d_ctrl)
    leaves_per_rank = 1 << (args.log_domain)
    out = torch.empty(leaves_per_rank * 8, dtype=torch.uint8, device=dev)
    desc = H.value_desc([(H.LEAF_INT, 64, 0)], True, 2, 1)
    # kPrgKeyLeft/Right/Value as uint128 (distributed_point_function.cc:37-42)
    keys = (int.from_bytes(bytes.fromhex("5be037ccf6a03de5935f08d0a5b6a2fd"), "big"),
            int.from_bytes(bytes.fromhex("ef94b6aedebb026ce2ea1fe0f66f4d0b"), "big"),
            int.from_bytes(bytes.fromhex("05a5d1588c5423e346a31101b21d1c98"), "big"))

    ev_k0, ev_k1 = [], []

    def step(timed_events=None):
        if k > 0:
            H.eval_paths(d_seed, d_ctrl, d_path, d_cws[:k], d_cl[:k], d_cr[:k], keys[0], keys[1],
                         seeds_out=sub_seed, ctrl_out=sub_ctrl, stream=stream)
            s0, c0 = sub_seed, sub_ctrl
        else:
            s0, c0 = d_seed, d_ctrl
        if timed_events is not None:
            timed_events[0].record(stream)
        H.expand(s0, c0, d_cws[k:], d_cl[k:], d_cr[k:], keys, desc, 2, d_vcw, 0, out=out,
                 stream=stream)
        if timed_events is not None:
            timed_events[1].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [(H.Event(), H.Event()) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    kern_ms = [a.elapsed_ms(b) for a, b in evs]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed * 1e3 / args.steps
    total_leaves = leaves_per_rank * world * args.steps
    value = total_leaves / elapsed
    kern_avg_ms = float(np.mean(kern_ms))
    aes_per_launch = 2 * (2**D - 1) + 1 * 2**D
    achieved = aes_per_launch / (kern_avg_ms * 1e-3) / 1e9
    bytes_per_launch = leaves_per_rank * 8
    if rank == 0:
        res = {
            "metric": "DPF leaf evals/sec, full-domain 2^30 uint64 at 1/2/4/8 GPUs; AES blocks/s",
            "value": value,
            "unit": "leaves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic key (random root seed, correction words, value correction)",
            "config": {"workload": f"full-domain EvaluateUntil, log_domain_size={log_domain}, "
                                   f"uint64, 2^{args.log_domain} leaves per GPU",
                       "log_domain_size": log_domain, "leaves_per_gpu": leaves_per_rank,
                       "tree_depth_per_gpu": D, "parallelism": f"subtree-prefix x{world}"},
            "aes_blocks_per_s": aes_per_launch * world * args.steps / elapsed,
            "roofline": {"bound": "valu", "achieved": achieved, "peak": AES_PEAK_GBLOCKS,
                         "unit": "G AES blocks/s", "frac": achieved / AES_PEAK_GBLOCKS,
                         "traffic": None, "kernel": "expand_kernel<FastIntLeaf<64,false>>",
                         "kernel_ms": kern_avg_ms,
                         "algorithmic_aes_per_launch": aes_per_launch},
            "roofline_hbm": {"bound": "hbm", "achieved": bytes_per_launch / (kern_avg_ms * 1e-3) / 1e9,
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": bytes_per_launch / (kern_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_sample_log, D_total)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
