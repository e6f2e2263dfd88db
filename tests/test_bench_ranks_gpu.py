"""bench.py's N-rank path on the GPU (the driver's scaling runs launch it as
`torch.distributed.run --nproc-per-node N bench.py --gpus N`).

RCCL refuses two ranks on one device, so DPF_BENCH_ONE_GPU=1 puts both ranks
on cuda:0 with a gloo group (bench.py: init_ranks): by default each rank
evaluates its 2^29-output half of config 2's one 2^30 domain (strong scaling,
the metric's configuration; no data-path collective), the barrier and the
max-over-ranks timing are the ones the 8-GPU run uses, and rank 0 prints one
line whose `value` counts the outputs of both ranks.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(extra):
    env = dict(os.environ, DPF_BENCH_ONE_GPU="1", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", *extra]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]   # rank 0 only
    return json.loads(lines[0])


def test_two_ranks_weak_scaling_line():
    d = _launch(["--scaling", "weak", "--log-domain", "26"])
    assert d["scaling"] == "weak"
    assert d["config"]["log_domain_size"] == 27 and d["config"]["outputs_per_gpu"] == 1 << 26


def test_two_ranks_on_one_gpu_strong_scaling_line():
    # The driver's N-GPU line: the metric's ONE 2^30 domain split over 2 ranks.
    d = _launch([])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1
    assert d["scaling"] == "strong"
    assert d["config"]["log_domain_size"] == 30
    assert d["config"]["outputs_per_gpu"] == 1 << 29
    assert d["roofline"]["sustained_clock_ghz"] > 0.5
    assert "api_level" not in d          # host output only in the one-GPU line
    pg = d["process_group"]
    assert pg["world_size"] == 2 and pg["backend"] == "gloo"
    assert len(pg["kernel_ms_per_rank"]) == 2
    # value = outputs of all ranks / max-over-ranks time of the timed steps.
    outputs = 2 * d["config"]["outputs_per_gpu"]
    assert d["value"] == pytest.approx(outputs / (d["ms_per_step"] * 1e-3), rel=1e-6)
    assert d["roofline"]["frac"] > 0


def test_unlaunched_gpus_flag_starts_n_ranks():
    # `python bench.py --gpus 2` with no launcher (the driver may call it that
    # way): bench.py starts the two ranks itself and relays rank 0's line.
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(DPF_BENCH_ONE_GPU="1", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--no-cpu-baseline", "--log-domain", "26"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["process_group"]["world_size"] == 2
    assert d["config"]["log_domain_size"] == 26 and d["config"]["outputs_per_gpu"] == 1 << 25


def test_unlaunched_gpus_beyond_visible_devices_fails():
    import torch
    n = torch.cuda.device_count() + 1
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "DPF_BENCH_ONE_GPU")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n),
                        "--steps", "1", "--warmup", "0", "--no-cpu-baseline"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and not r.stdout.strip()
    assert "visible" in r.stderr
