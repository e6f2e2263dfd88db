#!/usr/bin/env python3
"""Headline benchmark: full-domain DPF evaluation, 2^30 uint64 outputs per GPU.

Metric (BASELINE.json): "DPF leaf evals/sec, full-domain 2^30 uint64 at
1/2/4/8 GPUs; AES blocks/s" -- configs[1]: DpfParameters{log_domain_size=30,
value_type=uint64}, one key, EvaluateUntil(0, {}, ctx).

One *step* goes through the product API exactly as a caller would:
`DistributedPointFunction.evaluate_shard_to_device(0, rank, N, ctx, out)` on a
fresh EvaluationContext (the drop-in for EvaluateUntil(0, {}, ctx) with the
outputs left in HBM).  Inside it the host
library validates the context, uploads the correction words (a few KiB), and
launches the fused gfx950 expand kernel (ExpandSeeds + HashExpandedSeeds +
value correction) that writes 2^30 * 8 B = 8 GiB of corrected outputs to HBM.
Keys are generated on the CPU (out of scope for the GPU) before
the timed region.  The PCIe-inclusive host-output rate is a DESIGN.md note,
never `value`.

Multi-GPU (distributed_point_functions_amd/sharding.py): weak
scaling by subtree prefix.  With N = 2^k ranks the domain is 2^(30 + k); rank r
path-walks the top k tree levels along the bits of r and expands its own
2^30-output subtree.  No collective on the data path; one all_reduce(MAX) of
the step time outside the timed region.

Run: python bench.py [--gpus N --steps K --warmup W]
     python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

LOG_PER_GPU = 30          # 2^30 uint64 outputs per GPU (BASELINE.json configs[1])
AES_PEAK_GBLOCKS = 122.9  # integer-VALU AES-128 roofline (DESIGN.md "Roofline")
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md
METRIC = "DPF leaf evals/sec, full-domain 2^30 uint64 at 1/2/4/8 GPUs; AES blocks/s"
KERNEL = "expand_kernel<FastIntLeaf<64, false> >"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-domain", type=int, default=LOG_PER_GPU,
                    help="log2 outputs per GPU (default 30 = the BASELINE config)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-chunks", type=int, default=32,
                    help="CPU baseline sample = this many 2^24-output subtrees of the same key")
    return ap.parse_args()


def tree_aes_per_launch(depth: int, blocks_needed: int = 1) -> int:
    """AES-128 blocks one full-subtree expansion computes: two PRG calls per
    inner node (left/right children) plus `blocks_needed` value hashes per leaf
    seed."""
    return 2 * ((1 << depth) - 1) + blocks_needed * (1 << depth)


def cpu_baseline(key, log_domain: int, chunks: int):
    """The oracle (C restatement of dpf/distributed_point_function.cc:271-349,
    OpenSSL AES-NI in 64-block batches, one host thread) on a bounded sample of
    the SAME workload: `chunks` subtrees of 2^24 outputs of the benchmark key,
    each walked to its root (EvaluateSeeds) then expanded + hashed + corrected."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    P = O.OracleParams([(log_domain, ("int", 64), 0)])
    sub = 23                                  # 2^23 blocks = 2^24 uint64 outputs per chunk
    T = P.hierarchy_to_tree[0]
    top = T - sub
    # The product DpfKey (proto) restated as the oracle's key dict.
    k = {"seed": key.seed.high << 64 | key.seed.low, "party": key.party,
         "cws": [(c.seed.high << 64 | c.seed.low, int(c.control_left), int(c.control_right),
                  None) for c in key.correction_words],
         "last_vc": [[int(v.integer.value_uint64)] for v in key.last_level_value_correction]}
    vcw = O._value_correction(P, k, 0)
    cs_top, cl_top, cr_top = O._cw_arrays(k, 0, top)
    cs, cl, cr = O._cw_arrays(k, top, T)
    stride = (1 << top) // chunks
    leaves = 0
    t0 = time.perf_counter()
    for c in range(chunks):
        seed, ctrl = O.evaluate_seeds(O.blocks_from_ints([k["seed"]]),
                                      np.array([k["party"]], np.uint8),
                                      O.blocks_from_ints([c * stride]), cs_top, cl_top, cr_top)
        es, ec = O.expand_seeds(seed, ctrl, cs, cl, cr)
        out = O.hash_correct(("int", 64), es, ec, 1, P.cepb(0), vcw, k["party"])
        leaves += out.shape[0]
    dt = time.perf_counter() - t0
    return {"value": leaves / dt, "unit": "leaves/s", "cores": 1, "kind": "port",
            "sample": f"{chunks} subtrees x 2^24 uint64 outputs of the benchmark key "
                      f"(2^{log_domain} domain): EvaluateSeeds to each subtree root, then "
                      f"ExpandSeeds+HashExpandedSeeds+correction; {dt:.1f} s on 1 host thread",
            "aes_blocks_per_s": chunks * (tree_aes_per_launch(sub) + top) / dt}


def profiled_traffic(leaves_per_launch: int):
    """Per-launch HBM bytes of the dominant kernel from the newest committed
    rocprofv3 PMC summary for this workload (profiles/<round>_summary.json,
    FETCH_SIZE/WRITE_SIZE with the gfx950 corrections of MI355X_MICROARCH.md)."""
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_summary.json"))):
        try:
            s = json.load(open(f))
        except (OSError, ValueError):
            continue
        if s.get("leaves_per_launch") == leaves_per_launch and "hbm_traffic_bytes" in s:
            best = (s["hbm_traffic_bytes"], os.path.relpath(f, ROOT))
    return best


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from distributed_point_functions_amd import dpf as D
    from distributed_point_functions_amd import hip_abi as H
    from distributed_point_functions_amd import proto as pb
    from distributed_point_functions_amd import sharding as S

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    H.load(require_gpu=True)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)

    log_domain = S.weak_scaling_log_domain(args.log_domain, world)
    params = pb.DpfParameters()
    params.log_domain_size = log_domain
    params.value_type.CopyFrom(D.integer_type(64))
    dpf = D.DistributedPointFunction.create(params)
    # Same key on every rank: root seeds injected (GenerateKeysIncrementalWithSeeds).
    alpha = 0x2545F4914F6CDD1D % (1 << log_domain)
    beta = D.to_value(D.integer_type(64), 0xDEADBEEF)
    key, _ = dpf.generate_keys_incremental(alpha, [beta], seeds=(0x243F6A8885A308D3,
                                                                 0x13198A2E03707344))
    ctx0 = dpf.create_evaluation_context(key)
    depth = dpf.hierarchy_to_tree()[0] - S.shard_bits(world)   # tree levels expanded per rank
    outputs_per_rank = 1 << args.log_domain
    out = torch.empty(outputs_per_rank * 8, dtype=torch.uint8, device=dev)

    def step(evs=None):
        ctx = pb.EvaluationContext()
        ctx.CopyFrom(ctx0)
        if evs is not None:
            evs[0].record(stream)
        n = dpf.evaluate_shard_to_device(0, rank, world, ctx, out, stream=stream)
        if evs is not None:
            evs[1].record(stream)
        return n

    for _ in range(args.warmup):
        assert step() == outputs_per_rank
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
    kern_ms = float(np.mean([a.elapsed_ms(b) for a, b in evs]))
    elapsed = S.max_over_ranks(t1 - t0, device=dev if world > 1 else None)
    kern_ms_max = S.max_over_ranks(kern_ms, device=dev if world > 1 else None)

    # Spot-check the last step's output (sum of the two parties' shares is beta
    # at alpha, 0 elsewhere) on a few positions of this rank's shard.
    _check_shard(dpf, key, out, rank, world, outputs_per_rank, alpha)

    aes_per_launch = tree_aes_per_launch(depth)
    achieved = aes_per_launch / (kern_ms_max * 1e-3) / 1e9
    bytes_per_launch = outputs_per_rank * 8
    ms_per_step = elapsed * 1e3 / args.steps
    total = outputs_per_rank * world * args.steps
    if rank == 0:
        tr = profiled_traffic(outputs_per_rank)
        res = {
            "metric": METRIC,
            "value": total / elapsed,
            "unit": "leaves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: one DpfKey from the product keygen with fixed root seeds",
            "config": {"workload": f"full-domain EvaluateUntil(0, {{}}) of one key, "
                                   f"log_domain_size={log_domain}, uint64, 2^{args.log_domain} "
                                   f"outputs per GPU",
                       "log_domain_size": log_domain, "value_type": "uint64",
                       "outputs_per_gpu": outputs_per_rank, "tree_levels_per_gpu": depth,
                       "parallelism": f"subtree-prefix x{world}"},
            "aes_blocks_per_s": aes_per_launch * world * args.steps / elapsed,
            "roofline": {"bound": "valu", "achieved": achieved, "peak": AES_PEAK_GBLOCKS,
                         "unit": "G AES-128 blocks/s", "frac": achieved / AES_PEAK_GBLOCKS,
                         "traffic": tr[0] if tr else None,
                         "traffic_source": tr[1] if tr else None,
                         "kernel": KERNEL, "launch_ms": kern_ms_max,
                         "algorithmic_aes_per_launch": aes_per_launch,
                         "algorithmic_bytes_per_launch": bytes_per_launch},
            "roofline_hbm": {"bound": "hbm",
                             "achieved": bytes_per_launch / (kern_ms_max * 1e-3) / 1e9,
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": bytes_per_launch / (kern_ms_max * 1e-3) / 1e9 / HBM_PEAK_GBS},
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(key, log_domain, args.cpu_chunks)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _check_shard(dpf, key, out, rank, world, n, alpha):
    """EvaluateAt on a handful of points of this shard must equal the device
    output (cheap, outside the timed region)."""
    import torch
    rng = np.random.default_rng(rank)
    local = sorted({0, n - 1, *map(int, rng.integers(0, n, size=6))})
    if alpha // n == rank:
        local.append(alpha % n)
    words = out.view(torch.int64)
    pts = [rank * n + i for i in local]
    want = np.asarray(dpf.evaluate_at(key, 0, pts), dtype=np.uint64)
    got = np.array([int(words[i].item()) & (2**64 - 1) for i in local], dtype=np.uint64)
    if not np.array_equal(got, want):
        raise SystemExit(f"rank {rank}: device output disagrees with EvaluateAt at {pts}")


if __name__ == "__main__":
    main()
