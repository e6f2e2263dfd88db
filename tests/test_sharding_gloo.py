"""The multi-GPU partition (distributed_point_functions_amd.sharding) on CPU
ranks over gloo: each rank computes its subtree-prefix shard exactly the way
EvaluateShardToDevice does on a GPU (path-walk the top k levels, expand the
rest, hash + correct) -- here with the oracle -- and the gathered shards must
equal the oracle's full-domain EvaluateUntil.  Also covers max_over_ranks."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle as O
from distributed_point_functions_amd import sharding as S


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard_with_oracle(P, key, h, world, rank):
    """Oracle restatement of EvaluateShardToDevice for one rank."""
    k = S.shard_bits(world)
    stop = P.hierarchy_to_tree[h]
    seed = O.blocks_from_ints([key["seed"]])
    ctrl = np.array([key["party"]], np.uint8)
    if k:
        cs, cl, cr = O._cw_arrays(key, 0, k)
        seed, ctrl = O.evaluate_seeds(seed, ctrl, O.blocks_from_ints([rank]), cs, cl, cr)
    cs, cl, cr = O._cw_arrays(key, k, stop)
    es, ec = O.expand_seeds(seed, ctrl, cs, cl, cr)
    vt = P.vtypes[h]
    return O.hash_correct(vt, es, ec, P.blocks_needed[h], P.cepb(h),
                          O._value_correction(P, key, h), key["party"])


def _log_domain(scaling, log, world):
    """bench.py's domain: fixed (strong, the metric's configuration) or grown
    with the world (weak)."""
    return log if scaling == "strong" else S.weak_scaling_log_domain(log, world)


def _worker(rank, world, port, scaling, log, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        log_domain = _log_domain(scaling, log, world)
        P = O.OracleParams([(log_domain, ("int", 64), 0)])
        k0, k1 = O.generate_keys(P, 0x1234567 % (1 << log_domain), [[42]], 5, 6)
        res = {}
        for key in (k0, k1):
            mine = _shard_with_oracle(P, key, 0, world, rank)
            parts = [None] * world
            dist.all_gather_object(parts, mine)
            res[key["party"]] = parts
        t = S.max_over_ranks(float(rank) + 0.5)
        if rank == 0:
            q.put((res, t))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,scaling", [(2, "strong"), (4, "strong"), (8, "strong"),
                                           (2, "weak"), (4, "weak")])
def test_shards_concatenate_to_full_domain(world, scaling):
    # strong: one 2^12 domain split `world` ways (bench.py's default, the
    # metric's fixed-domain configuration); weak: 2^10 outputs per rank.
    log = 12 if scaling == "strong" else 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, scaling, log, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res, t = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert t == world - 0.5
    log_domain = _log_domain(scaling, log, world)
    per_rank = S.strong_scaling_log_outputs(log_domain, world)
    if scaling == "weak":
        assert per_rank == log
    P = O.OracleParams([(log_domain, ("int", 64), 0)])
    k0, k1 = O.generate_keys(P, 0x1234567 % (1 << log_domain), [[42]], 5, 6)
    for key in (k0, k1):
        full = O.evaluate_until(P, 0, [], O.create_context(P, key))
        parts = res[key["party"]]
        n = len(full)
        assert n == 1 << log_domain
        for r, part in enumerate(parts):
            a, b = S.shard_range(n, world, r)
            assert part.shape[0] == b - a == 1 << per_rank
        np.testing.assert_array_equal(np.concatenate(parts), full)


def test_partition_helpers():
    assert S.shard_bits(1) == 0 and S.shard_bits(8) == 3
    assert S.weak_scaling_log_domain(30, 8) == 33
    assert S.strong_scaling_log_outputs(30, 8) == 27
    assert S.strong_scaling_log_outputs(30, 1) == 30
    with pytest.raises(ValueError):
        S.strong_scaling_log_outputs(2, 8)
    assert S.shard_range(16, 4, 3) == (12, 16)
    for bad in (0, 3, 6):
        with pytest.raises(ValueError):
            S.shard_bits(bad)
    with pytest.raises(ValueError):
        S.shard_range(16, 4, 4)
    assert S.max_over_ranks(3.0) == 3.0


# ------------------------------------------------- key-batch sharding (config 4/5)
VTS = {"intmodn32x2": (("tuple", [("intmodn", 32, 4294967291)] * 2), [[1, 1]]),
       "u64": (("int", 64), [[3]]),
       "u16": (("int", 16), [[40000]]),
       "u128": (("int", 128), [[5]])}   # u128: the all-gather fallback


def _key_worker(rank, world, port, q, vt_name="intmodn32x2", device="cpu"):
    import torch
    import torch.distributed as dist
    from distributed_point_functions_amd import dpf as D
    from test_host_api_cpu import params, vt_from_oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        vt, beta = VTS[vt_name]
        levels = [(16, vt, 64.0)]
        P = O.OracleParams(levels)
        dpf = D.DistributedPointFunction.create_incremental(params(levels))
        dpf.register_value_type(vt_from_oracle(vt))
        n_keys, pts = 23, [0, 5, 77, 4095, 65535, 1234]
        rng = np.random.default_rng(17)          # same keys on every rank
        alphas = [int(a) for a in rng.integers(0, 1 << 16, size=n_keys)]
        keys = [O.generate_keys(P, a, beta, 1000 + k, 2000 + k)[k % 2]
                for k, a in enumerate(alphas)]
        lo, hi = S.key_range(n_keys, world, rank)
        part = None
        for k in range(lo, hi):
            v = O.evaluate_at(P, keys[k], 0, pts)
            part = v if part is None else O.add_packed(vt, part, v)
        if part is None:
            part = np.zeros((len(pts), O.packed_size(vt)), np.uint8)
        # device="cuda": the partial sums live in HBM as on a GPU rank; widening and
        # narrowing run there, only the gloo collective itself goes through host.
        packed = torch.from_numpy(part.reshape(-1).copy()).to(device)
        total = S.aggregate_shares(dpf, 0, packed, len(pts))
        if rank == 0:
            q.put(total)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _aggregate_case(world, vt_name, device="cpu"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_key_worker, args=(r, world, port, q, vt_name, device))
             for r in range(world)]
    for p in procs:
        p.start()
    total = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    vt, beta = VTS[vt_name]
    P = O.OracleParams([(16, vt, 64.0)])
    rng = np.random.default_rng(17)
    alphas = [int(a) for a in rng.integers(0, 1 << 16, size=23)]
    pts = [0, 5, 77, 4095, 65535, 1234]
    want = None
    for k, a in enumerate(alphas):
        v = O.evaluate_at(P, O.generate_keys(P, a, beta, 1000 + k, 2000 + k)[k % 2], 0, pts)
        want = v if want is None else O.add_packed(vt, want, v)
    np.testing.assert_array_equal(total.reshape(want.shape), want)


@pytest.mark.parametrize("world,vt_name", [(2, "intmodn32x2"), (3, "intmodn32x2"), (2, "u64"),
                                           (3, "u16"), (2, "u128")])
def test_key_batch_shards_aggregate_to_full_sum(world, vt_name):
    """all_reduce(SUM) of widened leaves (ints <= 64 bits, IntModN32) or the
    all-gather fallback (uint128) gives the sum over all keys."""
    _aggregate_case(world, vt_name)


@pytest.mark.gpu
@pytest.mark.parametrize("vt_name", ["intmodn32x2", "u64", "u128"])
def test_key_batch_aggregate_cuda_tensors(vt_name):
    """The same aggregation with the partial sums resident on cuda:0 (two gloo
    ranks share the card): the device-side widen/narrow code that an RCCL
    group runs, with only the backend differing."""
    _aggregate_case(2, vt_name, device="cuda:0")


def test_widen_narrow_roundtrip():
    """widen_leaves / narrow_leaves are exact inverses on reduced values, incl.
    a 64-bit leaf with the top bit set (wraps through int64)."""
    import torch
    leaves = [("int", 64, 0), ("intmodn", 32, 4294967291), ("int", 16, 0)]
    rng = np.random.default_rng(3)
    rows = np.zeros((5, 14), np.uint8)
    rows[:, 0:8] = rng.integers(0, 256, size=(5, 8), dtype=np.uint8)
    rows[0, 7] = 0xFF
    m = rng.integers(0, 4294967291, size=5, dtype=np.uint64)
    rows[:, 8:12] = m.astype("<u4").view(np.uint8).reshape(5, 4)
    rows[:, 12:14] = rng.integers(0, 256, size=(5, 2), dtype=np.uint8)
    packed = torch.from_numpy(rows.reshape(-1).copy())
    wide = S.widen_leaves(leaves, packed, 5)
    assert wide.dtype == torch.int64 and tuple(wide.shape) == (5, 3)
    assert int(wide[0, 0]) < 0                   # top bit set -> negative int64
    np.testing.assert_array_equal(S.narrow_leaves(leaves, wide, 5).numpy(), rows.reshape(-1))
    # doubling then narrowing = the group sum of a row with itself
    twice = S.narrow_leaves(leaves, wide * 2, 5).numpy().reshape(5, 14)
    lo = rows[:, 0:8].copy().view("<u8").reshape(5)
    np.testing.assert_array_equal(twice[:, 0:8].copy().view("<u8").reshape(5), lo * np.uint64(2))
    np.testing.assert_array_equal(twice[:, 8:12].copy().view("<u4").reshape(5),
                                  ((m * 2) % 4294967291).astype(np.uint32))


def test_key_range_partition():
    for n in (0, 1, 7, 1 << 20):
        for w in (1, 2, 3, 8):
            rs = [S.key_range(n, w, r) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
