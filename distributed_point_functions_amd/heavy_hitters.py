"""Multi-client heavy hitters over a 128-bit prefix hierarchy (SURVEY.md
config 5b) -- the caller of the incremental-evaluation path that the
reference's experiments/synthetic_data_benchmarks.cc exercises with one key.

Each of K clients holds a 128-bit value alpha_k and submits one DPF key pair
for the point function alpha_k -> beta over the hierarchy {8, 10, ..., 128}
with values Tuple<IntModN<uint32, N>, IntModN<uint32, N>> (N = 2^32 - 5,
security parameter 64 so the deep levels stay valid).  Server
p holds the p-th key of every client.  Level by level, both servers evaluate
ALL their keys at the current candidate prefixes and sum the shares over keys
(EvaluateUntil per key, distributed_point_function.h:641-837, batched on the
GPU with a device-resident context: DistributedPointFunction::
EvaluateUntilBatchSumToDevice).  Adding the two servers' sums reconstructs,
for every child of every candidate, (count, count * beta_1) mod N -- the
number of clients whose value starts with that child prefix.  The <= top_k
heaviest children with a nonzero count become the next level's candidates,
identically on every rank and both servers (the threshold step of the
two-server protocol, here run in one process).

Keys are split across ranks by client (sharding.key_range); each rank sums
over its own clients on the device and the per-rank sums are combined by one
all_reduce(SUM) of the widened IntModN32 leaves, reduced mod N on every rank
(sharding.aggregate_shares) -- the only data-path exchange,
<= top_k * 4 elements of 8 bytes per level and server.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import dpf as D
from . import proto as pb

MODULUS = 4294967291            # 2^32 - 5
SECURITY_PARAMETER = 64.0
BETA = (1, 7)                   # element 0 counts clients, element 1 = 7 * count


def value_type() -> pb.ValueType:
    m = D.int_mod_n_type(32, MODULUS)
    return D.tuple_type(m, m)


def hierarchy(first: int = 8, step: int = 2, last: int = 128) -> List[int]:
    logs = list(range(first, last + 1, step))
    if logs[-1] != last:
        logs.append(last)
    return logs


def parameters(logs: Sequence[int]) -> List[pb.DpfParameters]:
    out = []
    for log in logs:
        p = pb.DpfParameters()
        p.log_domain_size = log
        p.value_type.CopyFrom(value_type())
        p.security_parameter = SECURITY_PARAMETER
        out.append(p)
    return out


def create_dpf(logs: Sequence[int]):
    dpf = D.DistributedPointFunction.create_incremental(parameters(logs))
    dpf.register_value_type(value_type())
    return dpf


def client_values(num_clients: int, seed: int = 1, distinct: int = 1 << 14,
                  zipf_s: float = 1.1) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Synthetic client inputs: `distinct` random 128-bit values, client k holds
    value index idx[k] drawn from a Zipf(s) law truncated to `distinct` ranks.
    Returns (values (distinct, 2) uint64 {low, high}, idx (K,), alphas (K, 2))."""
    rng = np.random.default_rng(seed)
    values = rng.integers(0, 2**64, size=(distinct, 2), dtype=np.uint64)
    ranks = np.arange(1, distinct + 1, dtype=np.float64)
    p = ranks ** -zipf_s
    p /= p.sum()
    idx = rng.choice(distinct, size=num_clients, p=p)
    return values, idx, values[idx]


def plaintext_prefix_counts(values: np.ndarray, idx: np.ndarray, log: int,
                            top_log: int = 128) -> Dict[int, int]:
    """Number of clients per `log`-bit prefix of their `top_log`-bit values
    (the verification reference)."""
    per_value = np.bincount(idx, minlength=values.shape[0])
    out: Dict[int, int] = {}
    for (lo, hi), c in zip(values.tolist(), per_value.tolist()):
        if c:
            v = ((int(hi) << 64) | int(lo)) >> (top_log - log)
            out[v] = out.get(v, 0) + c
    return out


class Server:
    """One server's device state: its key shard, batch context and output."""

    def __init__(self, dpf, device_batch, max_outputs: int, device):
        import torch
        self.dpf = dpf
        self.keys = device_batch
        self.ctx = dpf.create_batch_evaluation_context(device_batch)
        self.out = torch.empty(max_outputs * 8, dtype=torch.uint8, device=device)

    def reset(self) -> None:
        """Restarts at the first level; keeps the expansion cache's buffers."""
        self.ctx.reset()

    def release_expansion_cache(self) -> None:
        self.ctx.release_expansion_cache()

    def evaluate(self, level: int, prefixes: Sequence[int], stream=None) -> int:
        return self.dpf.evaluate_until_batch_to_device(level, prefixes, self.ctx, self.out,
                                                       sum_over_keys=True, stream=stream)


def output_values(prefixes: Sequence[int], step: int, n: int) -> List[int]:
    """Domain values of a level's outputs: child r of prefix i is output
    i * 2^step + r (the reference's output order, h:817-836)."""
    if not prefixes:
        return list(range(n))
    cnt = 1 << step
    return [(p << step) | r for p in prefixes for r in range(cnt)]


def select(values: Sequence[int], counts: np.ndarray, top_k: int) -> List[int]:
    """The <= top_k heaviest values with a nonzero count (ties: smaller value
    first), returned in ascending order."""
    nz = np.nonzero(counts)[0]
    order = sorted(nz.tolist(), key=lambda j: (-int(counts[j]), values[j]))
    return sorted(values[j] for j in order[:top_k])


def run(dpf, servers: Sequence[Server], logs: Sequence[int], top_k: int = 1024,
        aggregate: Optional[Callable] = None, stream=None,
        record: Optional[list] = None, keep_cache: bool = False) -> List[int]:
    """One full heavy-hitters pass over every hierarchy level.  `aggregate(level,
    packed_tensor, n)` combines per-rank sums (default: single rank).
    Returns the final candidates; appends (level, values, counts, tags) to
    `record` when given.  The servers' expansion caches (up to 64 GiB per
    buffer at 2^20 clients) are given back after the last level unless
    `keep_cache` -- a caller running pass after pass keeps them (regrowing
    them costs seconds per pass) and releases them itself afterwards."""
    prefixes: List[int] = []
    for h, log in enumerate(logs):
        step = log - (logs[h - 1] if h else 0)
        sums = []
        for srv in servers:
            n = srv.evaluate(h, prefixes, stream)
            part = srv.out[: n * 8]
            if aggregate is not None:
                sums.append(np.asarray(aggregate(h, part, n)).reshape(-1).view(np.uint32))
            else:
                sums.append(part.cpu().numpy().view(np.uint32))
        tot = np.zeros(sums[0].shape, dtype=np.uint64)
        for s in sums:
            tot = (tot + s.astype(np.uint64)) % MODULUS
        tot = tot.reshape(-1, 2)
        values = output_values(prefixes, step, tot.shape[0])
        counts = tot[:, 0]
        if record is not None:
            record.append((h, values, counts.copy(), tot[:, 1].copy()))
        prefixes = select(values, counts, top_k)
    if not keep_cache:
        for srv in servers:
            release = getattr(srv, "release_expansion_cache", None)
            if release is not None:
                release()
    return prefixes  # the heavy hitters of the last level


def verify(record, logs: Sequence[int], values: np.ndarray, idx: np.ndarray) -> None:
    """Every reconstructed (count, 7 * count) must match the plaintext."""
    for h, vals, counts, tags in record:
        ref = plaintext_prefix_counts(values, idx, logs[h], logs[-1])
        for v, c, t in zip(vals, counts.tolist(), tags.tolist()):
            want = ref.get(v, 0)
            if c != want or t != (BETA[1] * want) % MODULUS:
                raise AssertionError(f"level {h} (log {logs[h]}): prefix {v:#x} reconstructs "
                                     f"({c}, {t}), plaintext count {want}")


def algorithmic_aes(dpf, logs: Sequence[int], record, num_keys: int, walk: bool = True) -> int:
    """AES blocks one server spends per pass: per level with P
    prefixes, P*(D_p - D_pp) path steps (from the root at the second level) +
    2*P*(2^(D_h - D_p) - 1) expansion + b*P*2^(D_h - D_p) value hashes, with
    b = 2 blocks read by the sampling; the first level is a full expansion.
    walk=False: the device context's expansion cache supplies every level's
    tree nodes, so the path steps are not computed."""
    h2t = dpf.hierarchy_to_tree()
    total = 0
    for h, vals, _, _ in record:
        d_h = h2t[h]
        if h == 0:
            total += 2 * ((1 << d_h) - 1) + 2 * (1 << d_h)
            continue
        p = len(vals) >> (logs[h] - logs[h - 1])
        d_p = h2t[h - 1]
        steps = d_p - (h2t[h - 2] if h >= 2 else 0) if walk else 0
        total += p * steps + 2 * p * ((1 << (d_h - d_p)) - 1) + 2 * p * (1 << (d_h - d_p))
    return total * num_keys
