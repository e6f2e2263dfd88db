#!/usr/bin/env python3
"""Same-box A/B of the full-domain expand kernel at config 2 (one start seed,
29 levels, uint64, 2^30 outputs, random correction words: timing only, parity
is the tests' job).  Each variant is `lib[:ENV=V,ENV=V]` and runs in its own
process, alternating variants over `--rounds` passes; prints one JSON line per
run with the mean of `--reps` HIP-event-timed launches.

  python tools/expand_ab.py --variants distributed_point_functions_amd/lib/libdpf_hip.so \\
      'distributed_point_functions_amd/lib/libdpf_hip.so:DPF_EXPAND_WS=0'
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


VALUES = {  # name: (leaves, elements per block, packed bytes per element[, blocks needed, direct])
    "u64": ([(0, 64, 0)], 2, 8),
    "t32_64": ([(0, 32, 0), (0, 64, 0)], 1, 12),   # Tuple<uint32_t, uint64_t>: SwarLeaf
    "t16x3": ([(0, 16, 0)] * 3, 2, 6),             # Tuple<uint16_t x 3>: uniform lanes
    # Tuple<IntModN<uint32_t, 2^32 - 5> x 2>: Mod32Leaf, two value blocks per leaf
    "m32x2": ([(1, 32, 4294967291)] * 2, 1, 8, 2, False),
}


def run_one(reps, levels, starts, value="u64"):
    import numpy as np
    import torch
    from distributed_point_functions_amd import hip_abi as H
    H.load(require_gpu=True)
    dev = torch.device("cuda")
    s = torch.cuda.current_stream()
    g = torch.Generator(device=dev)
    g.manual_seed(7)

    def rand_blocks(n):
        return torch.randint(-2**63, 2**63 - 1, (n, 2), dtype=torch.int64, device=dev, generator=g)

    keys = (0x5be037ccf6a03de5935f08d0a5b6a2fd, 0xef94b6aedebb026ce2ea1fe0f66f4d0b,
            0x05a5d1588c5423e346a31101b21d1c98)
    leaves, epb, esz, *rest = VALUES[value]
    bn = rest[0] if rest else 1
    desc = H.value_desc(leaves, rest[1] if len(rest) > 1 else True, epb, bn)
    D = levels
    seeds = rand_blocks(starts)
    ctrl = torch.zeros(starts, dtype=torch.uint8, device=dev)
    cws = rand_blocks(D)
    cl = torch.randint(0, 2, (D,), dtype=torch.uint8, device=dev, generator=g)
    cr = torch.randint(0, 2, (D,), dtype=torch.uint8, device=dev, generator=g)
    vcw = rand_blocks(epb * len(leaves))
    out = torch.empty(starts * (1 << D) * epb * esz, dtype=torch.uint8, device=dev)
    fn = lambda: H.expand(seeds, ctrl, cws, cl, cr, keys, desc, epb, vcw, 0, out=out)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    ev = [(H.Event(), H.Event()) for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    ms = [a.elapsed_ms(b) for a, b in ev]
    aes = starts * (2 * (2**D - 1) + bn * 2**D)
    print(json.dumps({"ms_mean": float(np.mean(ms)), "ms_min": float(np.min(ms)),
                      "gaes": aes / float(np.mean(ms)) / 1e6}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="*", default=[])
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--levels", type=int, default=29)
    ap.add_argument("--starts", type=int, default=1)
    ap.add_argument("--value", default="u64", choices=sorted(VALUES))
    ap.add_argument("--one", action="store_true")
    a = ap.parse_args()
    if a.one:
        return run_one(a.reps, a.levels, a.starts, a.value)
    for _ in range(a.rounds):
        for v in a.variants:
            lib, _, envs = v.partition(":")
            env = dict(os.environ, DPF_HIP_LIB=os.path.abspath(lib))
            for kv in filter(None, envs.split(",")):
                k, _, val = kv.partition("=")
                env[k] = val
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", "--reps",
                                str(a.reps), "--levels", str(a.levels), "--starts", str(a.starts),
                                "--value", a.value],
                               env=env, capture_output=True, text=True, timeout=300)
            for line in r.stdout.splitlines():
                if line.startswith("{"):
                    d = json.loads(line)
                    d["variant"] = v
                    print(json.dumps(d), flush=True)
                elif line.startswith("ws "):
                    print(f"  [{v}] {line}", flush=True)
            if r.returncode:
                print(f"  [{v}] rc={r.returncode}: {r.stderr[-2000:]}", flush=True)
                return r.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
