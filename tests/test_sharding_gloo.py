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


def _worker(rank, world, port, log_per_gpu, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        log_domain = S.weak_scaling_log_domain(log_per_gpu, world)
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


@pytest.mark.parametrize("world", [2, 4])
def test_shards_concatenate_to_full_domain(world):
    log_per_gpu = 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, log_per_gpu, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res, t = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert t == world - 0.5
    log_domain = S.weak_scaling_log_domain(log_per_gpu, world)
    P = O.OracleParams([(log_domain, ("int", 64), 0)])
    k0, k1 = O.generate_keys(P, 0x1234567 % (1 << log_domain), [[42]], 5, 6)
    for key in (k0, k1):
        full = O.evaluate_until(P, 0, [], O.create_context(P, key))
        parts = res[key["party"]]
        n = len(full)
        for r, part in enumerate(parts):
            a, b = S.shard_range(n, world, r)
            assert part.shape[0] == b - a == 1 << log_per_gpu
        np.testing.assert_array_equal(np.concatenate(parts), full)


def test_partition_helpers():
    assert S.shard_bits(1) == 0 and S.shard_bits(8) == 3
    assert S.weak_scaling_log_domain(30, 8) == 33
    assert S.shard_range(16, 4, 3) == (12, 16)
    for bad in (0, 3, 6):
        with pytest.raises(ValueError):
            S.shard_bits(bad)
    with pytest.raises(ValueError):
        S.shard_range(16, 4, 4)
    assert S.max_over_ranks(3.0) == 3.0
