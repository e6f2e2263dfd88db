"""RCCL on a one-GPU box: the N-rank path's collectives in a world-size-1
NCCL (= RCCL on ROCm) process group, so the driver's first 8-GPU run does not
also debut this code.

* `sharding.all_reduce_shares` -- the widen / all_reduce(SUM) / narrow of the
  per-rank share sums (configs 4 and 5b) -- on CUDA tensors under `nccl`;
* the max-over-ranks timing and the per-rank gathers on CUDA scalars;
* `bench.py` itself with DPF_BENCH_FORCE_PG=1: `init_process_group("nccl",
  device_id=...)`, its barriers, the timing collectives and (evaluate_at_sum,
  heavy_hitters) the share aggregation through RCCL.

Each case runs in a subprocess of its own: a process group is process state.
"""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "DPF_BENCH_ONE_GPU")}
    env.update(PYTHONUNBUFFERED="1", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


SCRIPT = textwrap.dedent("""
    import sys
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, {root!r})
    from distributed_point_functions_amd import sharding as S

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    rng = np.random.default_rng(7)
    N = 4294967291
    cases = {{
        "u64": [("int", 64, 0)],
        "intmodn32x2": [("intmodn", 32, N), ("intmodn", 32, N)],
        "u32_u16": [("int", 32, 0), ("int", 16, 0)],
    }}
    for name, leaves in cases.items():
        count = 1000
        width = sum(b // 8 for _, b, _ in leaves)
        raw = rng.integers(0, 256, size=count * width, dtype=np.uint8)
        # IntModN shares are < N: clear the top bit of every IntModN leaf.
        rows = raw.reshape(count, width)
        off = 0
        for kind, bits, _ in leaves:
            if kind == "intmodn":
                rows[:, off + bits // 8 - 1] &= 0x7F
            off += bits // 8
        packed = torch.from_numpy(raw.copy()).to(dev)
        wide = S.widen_leaves(leaves, packed, count)
        assert wide.is_cuda
        got = S.all_reduce_shares(leaves, packed, count)        # RCCL all_reduce(SUM)
        assert np.array_equal(got, raw), name                    # one rank: the identity
    t = S.max_over_ranks(2.5, device=dev)                        # RCCL all_reduce(MAX)
    assert t == 2.5
    assert S.gather_over_ranks(1.25, device=dev) == [1.25]       # RCCL all_gather
    g = S.all_gather_shares(torch.arange(16, dtype=torch.uint8, device=dev))
    assert g.shape == (1, 16) and g[0, 5] == 5
    info = S.group_info(3.0, device=dev)
    assert info["world_size"] == 1 and info["backend"] == "nccl"
    dist.barrier()
    dist.destroy_process_group()
    print("RCCL_OK")
""")


def test_share_collectives_through_rccl():
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(root=ROOT)], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "RCCL_OK" in r.stdout


@pytest.mark.parametrize("argv", [
    ["--workload", "full_domain", "--log-domain", "24", "--steps", "3", "--warmup", "1"],
    ["--workload", "evaluate_at_sum", "--keys-log", "12", "--points-log", "6", "--steps", "2",
     "--warmup", "1"],
    ["--workload", "heavy_hitters", "--keys-log", "10", "--top-k", "64"],
], ids=["full_domain", "evaluate_at_sum", "heavy_hitters"])
def test_bench_in_a_one_rank_rccl_group(argv):
    env = _env()
    env["DPF_BENCH_FORCE_PG"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1",
                        "--no-cpu-baseline", "--no-host-output", *argv],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    pg = d["process_group"]
    assert pg["world_size"] == 1 and pg["backend"] == "nccl"
    assert d["value"] > 0
