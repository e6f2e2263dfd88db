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

Strong scaling (bench.py's default, the metric's configuration: one 2^30
domain at 1/2/4/8 GPUs): the domain stays 2^log_domain and each rank
evaluates 2^(log_domain - k) outputs.  Weak scaling (`--scaling weak`, and
config 3's uint128 default): every rank keeps 2^log_per_gpu outputs, so the
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


def strong_scaling_log_outputs(log_domain: int, world: int) -> int:
    """log2 of the outputs each of `world` ranks evaluates of one 2^log_domain domain."""
    k = shard_bits(world)
    if k > log_domain:
        raise ValueError(f"{world} shards of a 2^{log_domain} domain")
    return log_domain - k


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
    identity without an initialised group (a one-rank group still runs the
    collective, so the RCCL path is exercised on a one-GPU box)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64,
                     device=device if device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_over_ranks(value: float, device=None) -> list:
    """Every rank's value of a per-rank scalar, in rank order ([value] without
    an initialised group)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return [float(value)]
    t = torch.tensor([float(value)], dtype=torch.float64,
                     device=device if device is not None else "cpu")
    parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t)
    return [float(p.item()) for p in parts]


def group_info(kernel_ms: float, device=None) -> dict:
    """What the process group actually was (world size, backend) and the
    per-rank dominant-kernel time, for the bench line of every workload."""
    import torch.distributed as dist
    up = dist.is_available() and dist.is_initialized()
    per_rank = gather_over_ranks(kernel_ms, device)
    return {"world_size": dist.get_world_size() if up else 1,
            "backend": dist.get_backend() if up else None,
            "kernel_ms_min": min(per_rank), "kernel_ms_max": max(per_rank),
            "kernel_ms_per_rank": per_rank}


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
    if not (dist.is_available() and dist.is_initialized()):
        return packed.cpu().numpy().reshape(1, -1)
    if packed.is_cuda and dist.get_backend() == "gloo":
        packed = packed.cpu()   # gloo all-gathers host tensors only
    parts = [torch.empty_like(packed) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, packed.contiguous())
    return np.stack([p.cpu().numpy().reshape(-1) for p in parts])


def _widenable(leaves) -> bool:
    return all((kind == "int" and bits <= 64) or (kind == "intmodn" and 0 < mod <= (1 << 32))
               for kind, bits, mod in leaves)


def widen_leaves(leaves, packed, count: int):
    """[count, num_leaves] int64 tensor of the packed little-endian leaves, built
    on the tensor's own device (no host round trip): bytes shifted into place
    and summed (disjoint bit fields, so the sum is the OR; a 64-bit leaf's top
    byte wraps into the sign bit, which is exact mod 2^64)."""
    import torch
    rows = packed.reshape(count, -1)
    cols, off = [], 0
    for kind, bits, mod in leaves:
        w = bits // 8
        field = rows[:, off:off + w].to(torch.int64)
        shifts = torch.arange(0, 8 * w, 8, dtype=torch.int64, device=rows.device)
        cols.append((field << shifts).sum(dim=1))
        off += w
    return torch.stack(cols, dim=1)


def narrow_leaves(leaves, wide, count: int):
    """Inverse of widen_leaves after the group reduction: each int64 column
    reduced mod 2^bits or mod N (IntModN) and packed back into bytes."""
    import torch
    parts = []
    for i, (kind, bits, mod) in enumerate(leaves):
        v = wide[:, i]
        if kind == "intmodn":
            v = torch.remainder(v, mod)     # sums of < 2^31 values < 2^32 stay positive
        w = bits // 8
        shifts = torch.arange(0, 8 * w, 8, dtype=torch.int64, device=v.device)
        parts.append(((v.unsqueeze(1) >> shifts) & 0xFF).to(torch.uint8))
    return torch.cat(parts, dim=1).reshape(-1)


def all_reduce_shares(leaves, packed, count: int):
    """Group sum over ranks via one all_reduce(SUM) of the int64-widened leaves
    (requires _widenable(leaves)).  `packed` is a uint8 tensor on any device;
    widening, the collective (RCCL when the tensor is on a GPU and the group is
    NCCL) and the reduction mod 2^bits / N all run on that device, and only the
    packed result is copied to the host.  A gloo group moves the widened
    [count, leaves] int64 tensor to the host for the collective, nothing else
    differs.  Returns the packed host array."""
    import numpy as np
    import torch
    import torch.distributed as dist
    if not hasattr(packed, "reshape") or isinstance(packed, np.ndarray):
        packed = torch.from_numpy(np.ascontiguousarray(np.asarray(packed, np.uint8)))
    wide = widen_leaves(leaves, packed, count)
    if wide.is_cuda and dist.get_backend() == "gloo":
        wide = wide.cpu()   # gloo reduces host tensors only
    dist.all_reduce(wide, op=dist.ReduceOp.SUM)
    return narrow_leaves(leaves, wide.to(packed.device), count).cpu().numpy()


def aggregate_shares(dpf, hierarchy_level: int, packed, count: int):
    """Group sum over ranks of `count`-element packed partial sums: the
    cross-GPU step of the aggregation variant."""
    import torch.distributed as dist
    from . import dpf as D
    leaves = D.leaves_of(dpf.parameters()[hierarchy_level].value_type)
    if dist.is_available() and dist.is_initialized() and _widenable(leaves):
        return all_reduce_shares(leaves, packed, count)
    stacked = all_gather_shares(packed)
    return dpf.sum_packed_shares(hierarchy_level, stacked, stacked.shape[0], count)
