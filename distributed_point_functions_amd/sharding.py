"""Multi-GPU partition of a full-domain DPF level.

The reference evaluates one key on one host (`EvaluateUntil`,
dpf/distributed_point_function.h:785-835).  Full-domain evaluation is a tree
expansion whose subtrees are independent, so N GPUs split it by *subtree
prefix*: with N = 2^k ranks, rank r path-walks the top k tree levels along
the bits of r (MSB first, as `EvaluateSeeds` walks a path,
dpf/internal/evaluate_prg_hwy.cc:495-506) and expands the 2^(T-k)-leaf
subtree below it (`DistributedPointFunction::EvaluateShardToDevice`).  Shard r
covers output elements [r * n / N, (r + 1) * n / N): concatenating the shards
in rank order is the reference's full-domain output.  There is no exchange on
the data path; the only collective is the max-over-ranks of the step time.

Weak scaling (bench.py): every rank keeps 2^log_per_gpu outputs, so the
domain grows to 2^(log_per_gpu + k) with N.
"""
from __future__ import annotations


def shard_bits(world: int) -> int:
    """k = log2(world); the partition needs a power-of-two rank count."""
    if world < 1 or world & (world - 1):
        raise ValueError(f"world size must be a power of two, got {world}")
    return world.bit_length() - 1


def weak_scaling_log_domain(log_per_gpu: int, world: int) -> int:
    """Domain size (log2) that gives each of `world` ranks 2^log_per_gpu outputs."""
    return log_per_gpu + shard_bits(world)


def shard_range(num_outputs: int, world: int, rank: int) -> tuple:
    """[start, stop) of the output elements rank `rank` produces."""
    shard_bits(world)
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    if num_outputs % world:
        raise ValueError("output count not divisible by the shard count")
    per = num_outputs // world
    return rank * per, (rank + 1) * per


def max_over_ranks(value: float, device=None) -> float:
    """Max of a per-rank scalar (the step time) over the process group; the
    identity without an initialised group."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64,
                     device=device if device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ---------------------------------------------------------------------------
# Key-batch sharding (configs 4 and 5)
# ---------------------------------------------------------------------------
# Batched EvaluateAt and heavy-hitters aggregation over K keys split the keys
# into `world` contiguous row ranges (DeviceKeyBatch.upload(begin, end)).
# Per-key outputs stay on their rank; the aggregation variant reduces over the
# rank's keys on the device (dpf_hip_eval_points_sum) and then combines the
# per-rank partial sums -- the only data-path exchange, a few KiB over xGMI:
# * value types whose leaves are integers of <= 64 bits or IntModN with
#   N <= 2^32 (uint64 of config 4, Tuple<IntModN32, IntModN32> of config 5b):
#   each leaf widened to int64, ONE all_reduce(SUM) (RCCL), then reduced mod
#   2^bits or mod N locally (at most 2^31 ranks keep an IntModN32
#   sum inside int64);
# * anything else (uint128, IntModN over 64-bit bases, XorWrapper): one
#   all_gather of the packed sums and the group sum on every rank.

def key_range(num_keys: int, world: int, rank: int) -> tuple:
    """[begin, end) of the keys rank `rank` owns (balanced contiguous split)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    return num_keys * rank // world, num_keys * (rank + 1) // world


def all_gather_shares(packed):
    """All-gathers one rank's packed partial sums (a uint8 torch tensor, CPU for
    gloo or CUDA for RCCL) and returns the stacked [world, bytes] host array."""
    import numpy as np
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return packed.cpu().numpy().reshape(1, -1)
    if packed.is_cuda and dist.get_backend() == "gloo":
        packed = packed.cpu()   # gloo all-gathers host tensors only
    parts = [torch.empty_like(packed) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, packed.contiguous())
    return np.stack([p.cpu().numpy().reshape(-1) for p in parts])


def _widenable(leaves) -> bool:
    return all((kind == "int" and bits <= 64) or (kind == "intmodn" and 0 < mod <= (1 << 32))
               for kind, bits, mod in leaves)


def all_reduce_shares(leaves, packed, count: int):
    """Group sum over ranks via one all_reduce(SUM) of the int64-widened leaves
    (requires _widenable(leaves)); returns the packed host array."""
    import numpy as np
    import torch
    import torch.distributed as dist
    host = packed.cpu().numpy().reshape(count, -1) if hasattr(packed, "cpu") else \
        np.asarray(packed, np.uint8).reshape(count, -1)
    cols, off = [], 0
    for kind, bits, mod in leaves:
        w = bits // 8
        raw = np.ascontiguousarray(host[:, off:off + w]).view(f"<u{w}").reshape(count)
        cols.append(raw.astype(np.uint64).view(np.int64))
        off += w
    wide = torch.from_numpy(np.stack(cols, axis=1))
    dev = packed.device if (hasattr(packed, "is_cuda") and packed.is_cuda
                            and dist.get_backend() != "gloo") else torch.device("cpu")
    wide = wide.to(dev)
    dist.all_reduce(wide, op=dist.ReduceOp.SUM)
    total = wide.cpu().numpy().view(np.uint64)
    out = np.empty_like(host)
    off = 0
    for i, (kind, bits, mod) in enumerate(leaves):
        w = bits // 8
        v = total[:, i]
        v = v % np.uint64(mod) if kind == "intmodn" else (
            v & np.uint64((1 << bits) - 1) if bits < 64 else v)
        out[:, off:off + w] = v.astype(f"<u{w}").view(np.uint8).reshape(count, w)
        off += w
    return out.reshape(-1)


def aggregate_shares(dpf, hierarchy_level: int, packed, count: int):
    """Group sum over ranks of `count`-element packed partial sums: the
    cross-GPU step of the aggregation variant."""
    import torch.distributed as dist
    from . import dpf as D
    leaves = D.leaves_of(dpf.parameters()[hierarchy_level].value_type)
    if (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
            and _widenable(leaves)):
        return all_reduce_shares(leaves, packed, count)
    stacked = all_gather_shares(packed)
    return dpf.sum_packed_shares(hierarchy_level, stacked, stacked.shape[0], count)
